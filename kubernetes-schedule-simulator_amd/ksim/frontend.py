"""ctypes view of the C++ Kubernetes-field front end (include/ksim_k8s.h, csrc/ksim_k8s.cpp).

What a cgo adapter does in Go, done here from Kubernetes-shaped dicts: flatten v1.Node / v1.Pod /
PV / PVC / StorageClass objects into the ksim_k8s_* structs (quantities canonical — cpu as
MilliValue, the rest as Value — everything else as strings), hand them to libksim, and let the
library intern them and evaluate every scheduling string rule.  No rule is evaluated here: the
parity tests (tests/test_k8s_frontend.py) compare the library's tables with the Python host's
(ksim/ingest.py), and tests/c/ksim_c_loop.c drives the same entry points from plain C.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi, quantity

VOL_GCE_PD, VOL_EBS, VOL_AZURE_DISK, VOL_ISCSI, VOL_RBD, VOL_PVC, VOL_OTHER = 1, 2, 3, 4, 5, 6, 7
_CSTR = C.c_char_p


class KV(C.Structure):
    _fields_ = [("key", _CSTR), ("value", _CSTR)]


class Req(C.Structure):
    _fields_ = [("key", _CSTR), ("op", _CSTR), ("n_values", C.c_int32), ("values", C.POINTER(_CSTR))]


class NodeTerm(C.Structure):
    _fields_ = [("n_reqs", C.c_int32), ("reqs", C.POINTER(Req))]


class PrefNodeTerm(C.Structure):
    _fields_ = [("weight", C.c_int32), ("preference", NodeTerm)]


class LabelSelector(C.Structure):
    _fields_ = [("present", C.c_int32), ("n_match_labels", C.c_int32), ("match_labels", C.POINTER(KV)),
                ("n_exprs", C.c_int32), ("exprs", C.POINTER(Req))]


class PodTerm(C.Structure):
    _fields_ = [("selector", LabelSelector), ("n_namespaces", C.c_int32), ("namespaces", C.POINTER(_CSTR)),
                ("topology_key", _CSTR), ("weight", C.c_int32)]


class Taint(C.Structure):
    _fields_ = [("key", _CSTR), ("value", _CSTR), ("effect", _CSTR)]


class Toleration(C.Structure):
    _fields_ = [("key", _CSTR), ("op", _CSTR), ("value", _CSTR), ("effect", _CSTR)]


class Resource(C.Structure):
    _fields_ = [("name", _CSTR), ("value", C.c_int64)]


class Port(C.Structure):
    _fields_ = [("host_ip", _CSTR), ("protocol", _CSTR), ("host_port", C.c_int32)]


class Container(C.Structure):
    _fields_ = [("has_cpu", C.c_int32), ("has_mem", C.c_int32), ("cpu_milli", C.c_int64), ("mem", C.c_int64),
                ("gpu", C.c_int64), ("eph", C.c_int64), ("n_other", C.c_int32), ("other", C.POINTER(Resource)),
                ("qos_positive", C.c_int32), ("n_ports", C.c_int32), ("ports", C.POINTER(Port)), ("image", _CSTR)]


class Volume(C.Structure):
    _fields_ = [("kind", C.c_int32), ("read_only", C.c_int32), ("id", _CSTR), ("pool", _CSTR), ("image", _CSTR),
                ("n_monitors", C.c_int32), ("monitors", C.POINTER(_CSTR))]


class Pod(C.Structure):
    _fields_ = [("name", _CSTR), ("namespace_", _CSTR), ("n_labels", C.c_int32), ("labels", C.POINTER(KV)),
                ("deleting", C.c_int32), ("node_name", _CSTR),
                ("n_containers", C.c_int32), ("containers", C.POINTER(Container)),
                ("n_init_containers", C.c_int32), ("init_containers", C.POINTER(Container)),
                ("n_node_selector", C.c_int32), ("node_selector", C.POINTER(KV)),
                ("has_node_affinity", C.c_int32), ("has_required", C.c_int32),
                ("n_required_terms", C.c_int32), ("required_terms", C.POINTER(NodeTerm)),
                ("n_preferred", C.c_int32), ("preferred", C.POINTER(PrefNodeTerm)),
                ("n_tolerations", C.c_int32), ("tolerations", C.POINTER(Toleration)),
                ("has_pod_affinity", C.c_int32), ("has_pod_anti_affinity", C.c_int32),
                ("n_affinity_required", C.c_int32), ("n_affinity_preferred", C.c_int32),
                ("n_anti_required", C.c_int32), ("n_anti_preferred", C.c_int32),
                ("affinity_required", C.POINTER(PodTerm)), ("affinity_preferred", C.POINTER(PodTerm)),
                ("anti_required", C.POINTER(PodTerm)), ("anti_preferred", C.POINTER(PodTerm)),
                ("n_volumes", C.c_int32), ("volumes", C.POINTER(Volume)),
                ("n_spread", C.c_int32), ("spread", C.POINTER(LabelSelector)), ("spread_set_selector", C.POINTER(C.c_int32)),
                ("avoid_ctrl_kind", _CSTR), ("avoid_ctrl_uid", _CSTR), ("uid", _CSTR)]


class Condition(C.Structure):
    _fields_ = [("type", _CSTR), ("status", _CSTR)]


class Avoid(C.Structure):
    _fields_ = [("has_controller", C.c_int32), ("kind", _CSTR), ("uid", _CSTR)]


class Image(C.Structure):
    _fields_ = [("n_names", C.c_int32), ("names", C.POINTER(_CSTR)), ("size_bytes", C.c_int64)]


class Node(C.Structure):
    _fields_ = [("name", _CSTR), ("n_labels", C.c_int32), ("labels", C.POINTER(KV)), ("n_taints", C.c_int32),
                ("taints", C.POINTER(Taint)), ("unschedulable", C.c_int32), ("n_conditions", C.c_int32),
                ("conditions", C.POINTER(Condition)), ("alloc_cpu_milli", C.c_int64), ("alloc_mem", C.c_int64),
                ("alloc_gpu", C.c_int64), ("alloc_eph", C.c_int64), ("alloc_pods", C.c_int64),
                ("n_alloc_other", C.c_int32), ("alloc_other", C.POINTER(Resource)),
                ("n_avoid", C.c_int32), ("avoid", C.POINTER(Avoid)), ("has_images", C.c_int32),
                ("n_images", C.c_int32), ("images", C.POINTER(Image))]


class PV(C.Structure):
    _fields_ = [("name", _CSTR), ("n_labels", C.c_int32), ("labels", C.POINTER(KV)), ("kind", C.c_int32),
                ("id", _CSTR), ("has_node_affinity", C.c_int32)]


class PVC(C.Structure):
    _fields_ = [("namespace_", _CSTR), ("name", _CSTR), ("volume_name", _CSTR), ("storage_class", _CSTR)]


class StorageClass(C.Structure):
    _fields_ = [("name", _CSTR), ("binding_mode", _CSTR)]


class Weights(C.Structure):
    _fields_ = [("prefer_avoid", C.c_int64), ("image_locality", C.c_int64)]


class LabelPriority(C.Structure):
    _fields_ = [("label", C.c_char_p), ("presence", C.c_int32), ("pad", C.c_int32), ("weight", C.c_int64)]


class PolicyArgs(C.Structure):
    """ksim_k8s_policy_args: a Policy's CheckNodeLabelPresence / CheckServiceAffinity arguments and
    labelPreference / serviceAntiAffinity (no selecting service) priorities."""
    _fields_ = [("n_presence_labels", C.c_int32), ("presence", C.c_int32), ("presence_labels", C.POINTER(C.c_char_p)),
                ("n_affinity_labels", C.c_int32), ("services_select_pods", C.c_int32),
                ("affinity_labels", C.POINTER(C.c_char_p)), ("n_label_priorities", C.c_int32),
                ("has_service_anti_affinity", C.c_int32), ("label_priorities", C.POINTER(LabelPriority))]


class CacheOptions(C.Structure):
    _fields_ = [("cfg", abi.Config), ("extra", Weights), ("hard_weight", C.c_int32), ("max_vols", C.c_int32 * 3),
                ("port_slots", C.c_int32), ("check_volume_binding", C.c_int32), ("pad", C.c_int32),
                ("policy", C.POINTER(PolicyArgs))]


def policy_args(keep, label_presence=None, service_affinity=None, label_priorities=(), services_select_pods=False):
    """ksim_k8s_policy_args from a Policy's arguments (arrays kept alive in `keep`): label_presence =
    (labels, presence), service_affinity = labels, label_priorities = [(label, presence, weight,
    is_service_anti_affinity)]."""
    def strs(xs):
        arr = (C.c_char_p * max(len(xs), 1))(*[x.encode() for x in xs])
        keep.append(arr)
        return C.cast(arr, C.POINTER(C.c_char_p))
    a = PolicyArgs()
    if label_presence is not None:
        a.n_presence_labels, a.presence = len(label_presence[0]), int(bool(label_presence[1]))
        a.presence_labels = strs(list(label_presence[0]))
    if service_affinity is not None:
        a.n_affinity_labels = len(service_affinity)
        a.affinity_labels = strs(list(service_affinity))
    a.services_select_pods = int(bool(services_select_pods))
    lp = (LabelPriority * max(len(label_priorities), 1))(*[LabelPriority(l.encode(), int(bool(pr)), 0, int(wt))
                                                           for l, pr, wt, _ in label_priorities])
    keep.append(lp)
    a.n_label_priorities = len(label_priorities)
    a.has_service_anti_affinity = int(any(saa for _, _, _, saa in label_priorities))
    a.label_priorities = C.cast(lp, C.POINTER(LabelPriority))
    keep.append(a)
    return a


class Options(C.Structure):
    _fields_ = [("hard_weight", C.c_int32), ("max_vols", C.c_int32 * 3), ("port_slots", C.c_int32),
                ("vol_slots", C.c_int32), ("image_locality", C.c_int32)]


class _Keep(list):
    """Keeps the ctypes buffers a flattened object points into alive."""

    def s(self, x):
        if x is None:
            return None
        b = str(x).encode()
        self.append(b)
        return b

    def arr(self, ctype, items):
        a = (ctype * max(len(items), 1))(*items)
        self.append(a)
        return len(items), C.cast(a, C.POINTER(ctype))

    def strs(self, vals):
        return self.arr(_CSTR, [self.s(v) for v in vals or []])


def _kvs(k, d):
    return k.arr(KV, [KV(k.s(a), k.s(b)) for a, b in (d or {}).items()])


def _reqs(k, exprs):
    out = []
    for e in exprs or []:
        n, vals = k.strs(e.get("values"))
        out.append(Req(k.s(e.get("key", "")), k.s(e.get("operator", "")), n, vals))
    return k.arr(Req, out)


def _label_selector(k, ps):
    if ps is None:
        return LabelSelector(0, 0, None, 0, None)
    n_ml, ml = _kvs(k, ps.get("matchLabels"))
    n_ex, ex = _reqs(k, ps.get("matchExpressions"))
    return LabelSelector(1, n_ml, ml, n_ex, ex)


def _pod_terms(k, terms, weighted):
    out = []
    for t in terms or []:
        w = int(t.get("weight", 0)) if weighted else 0
        term = (t.get("podAffinityTerm") or {}) if weighted else t
        n_ns, nss = k.strs(term.get("namespaces"))
        out.append(PodTerm(_label_selector(k, term.get("labelSelector")), n_ns, nss, k.s(term.get("topologyKey") or ""), w))
    return k.arr(PodTerm, out)


def _container(k, c):
    req = (c.get("resources") or {}).get("requests") or {}
    lim = (c.get("resources") or {}).get("limits") or {}
    other = [Resource(k.s(n), quantity.value(q)) for n, q in req.items()
             if n not in ("cpu", "memory", "alpha.kubernetes.io/nvidia-gpu", "ephemeral-storage", "pods")]
    n_other, p_other = k.arr(Resource, other)
    qos = any(n in ("cpu", "memory") and quantity.positive(q) for rl in (req, lim) for n, q in rl.items())
    ports = [Port(k.s(p.get("hostIP") or ""), k.s(p.get("protocol") or ""), int(p.get("hostPort") or 0))
             for p in c.get("ports") or []]
    n_ports, p_ports = k.arr(Port, ports)
    g = lambda n, milli=False: (quantity.milli_value(req[n]) if milli else quantity.value(req[n])) if n in req else 0
    return Container(int("cpu" in req), int("memory" in req), g("cpu", True), g("memory"),
                     g("alpha.kubernetes.io/nvidia-gpu"), g("ephemeral-storage"), n_other, p_other, int(qos), n_ports, p_ports,
                     k.s(c.get("image") or ""))


def _volume(k, v):
    for key, kind, field in (("gcePersistentDisk", VOL_GCE_PD, "pdName"), ("awsElasticBlockStore", VOL_EBS, "volumeID"),
                             ("azureDisk", VOL_AZURE_DISK, "diskName"), ("iscsi", VOL_ISCSI, "iqn"),
                             ("persistentVolumeClaim", VOL_PVC, "claimName")):
        src = v.get(key)
        if src is not None:
            return Volume(kind, int(bool(src.get("readOnly"))), k.s(src.get(field, "")), None, None, 0, None)
    rbd = v.get("rbd")
    if rbd is not None:
        n, mons = k.strs(rbd.get("monitors"))
        return Volume(VOL_RBD, int(bool(rbd.get("readOnly"))), None, k.s(rbd.get("pool", "")), k.s(rbd.get("image", "")), n, mons)
    return Volume(VOL_OTHER, 0, None, None, None, 0, None)


def spread_raw(listers, pod, services_only=False):
    """getSelectors over the listers (ksim/spread.py SpreadListers._selectors), as raw selectors:
    [(selector dict, set_selector)] — what a Go adapter's listers hand the front end."""
    from . import labels
    if not listers:
        return []
    md = pod.get("metadata") or {}
    ns, lab = md.get("namespace", ""), md.get("labels") or {}
    out = []
    for svc in listers.services:
        sel = (svc.get("spec") or {}).get("selector")
        if (svc.get("metadata") or {}).get("namespace", "") == ns and sel is not None and listers._set_selects(sel, lab):
            out.append(({"matchLabels": sel}, 1))
    if services_only or not lab:
        return out
    for rc in listers.rcs:
        sel = (rc.get("spec") or {}).get("selector") or {}
        if (rc.get("metadata") or {}).get("namespace", "") == ns and sel and listers._set_selects(sel, lab):
            out.append(({"matchLabels": sel}, 1))
    for objs in (listers.rss, listers.sss):
        found = []
        try:
            for o in objs:
                if (o.get("metadata") or {}).get("namespace", "") != ns:
                    continue
                raw = (o.get("spec") or {}).get("selector")
                sel = labels.from_label_selector(raw)
                if sel is labels.NOTHING or len(sel) == 0 or not labels.matches(sel, lab):
                    continue
                found.append((raw, 0))
        except labels.SelectorError:
            found = []
        out.extend(found)
    return out


def flatten_pod(k, p, spread=()):
    """A v1.Pod dict → ksim_k8s_pod (buffers kept alive by k)."""
    md, spec = p.get("metadata") or {}, p.get("spec") or {}
    n_lab, labs = _kvs(k, md.get("labels"))
    n_c, cs = k.arr(Container, [_container(k, c) for c in spec.get("containers") or []])
    n_i, ics = k.arr(Container, [_container(k, c) for c in spec.get("initContainers") or []])
    n_ns, nsel = _kvs(k, spec.get("nodeSelector"))
    aff = spec.get("affinity") or {}
    na = aff.get("nodeAffinity")
    req = (na or {}).get("requiredDuringSchedulingIgnoredDuringExecution")
    terms = [NodeTerm(*_reqs(k, t.get("matchExpressions"))) for t in ((req or {}).get("nodeSelectorTerms") or [])]
    n_rt, rts = k.arr(NodeTerm, terms)
    prefs = [PrefNodeTerm(int(t.get("weight", 0)), NodeTerm(*_reqs(k, (t.get("preference") or {}).get("matchExpressions"))))
             for t in (na or {}).get("preferredDuringSchedulingIgnoredDuringExecution") or []]
    n_pf, pfs = k.arr(PrefNodeTerm, prefs)
    tols = [Toleration(k.s(t.get("key") or ""), k.s(t.get("operator") or ""), k.s(t.get("value") or ""), k.s(t.get("effect") or ""))
            for t in spec.get("tolerations") or []]
    n_t, ts = k.arr(Toleration, tols)
    pa, pn = aff.get("podAffinity"), aff.get("podAntiAffinity")
    n_ar, ar = _pod_terms(k, (pa or {}).get("requiredDuringSchedulingIgnoredDuringExecution"), False)
    n_ap, ap = _pod_terms(k, (pa or {}).get("preferredDuringSchedulingIgnoredDuringExecution"), True)
    n_nr, nr = _pod_terms(k, (pn or {}).get("requiredDuringSchedulingIgnoredDuringExecution"), False)
    n_np, npf = _pod_terms(k, (pn or {}).get("preferredDuringSchedulingIgnoredDuringExecution"), True)
    n_v, vs = k.arr(Volume, [_volume(k, v) for v in spec.get("volumes") or []])
    n_sp, sps = k.arr(LabelSelector, [_label_selector(k, s) for s, _ in spread])
    _, spf = k.arr(C.c_int32, [f for _, f in spread])
    from .ingest import avoid_controller
    ctrl = avoid_controller(md)
    return Pod(k.s(md.get("name", "")), k.s(md.get("namespace", "")), n_lab, labs, int(md.get("deletionTimestamp") is not None),
               k.s(spec.get("nodeName") or ""), n_c, cs, n_i, ics, n_ns, nsel, int(na is not None), int(req is not None),
               n_rt, rts, n_pf, pfs, n_t, ts, int(pa is not None), int(pn is not None), n_ar, n_ap, n_nr, n_np, ar, ap, nr, npf,
               n_v, vs, n_sp, sps, spf, k.s(ctrl[0]) if ctrl else None, k.s(ctrl[1]) if ctrl else None,
               k.s(md.get("uid") or ""))


def flatten_node(k, x):
    """A v1.Node dict → ksim_k8s_node."""
    from .ingest import avoid_signatures
    md, spec, st = x.get("metadata") or {}, x.get("spec") or {}, x.get("status") or {}
    n_lab, labs = _kvs(k, md.get("labels"))
    taints = [Taint(k.s(t.get("key") or ""), k.s(t.get("value") or ""), k.s(t.get("effect") or "")) for t in spec.get("taints") or []]
    n_t, ts = k.arr(Taint, taints)
    conds = [Condition(k.s(c.get("type")), k.s(c.get("status"))) for c in st.get("conditions") or []]
    n_c, cs = k.arr(Condition, conds)
    al = st.get("allocatable") or {}
    g = lambda n, milli=False: (quantity.milli_value(al[n]) if milli else quantity.value(al[n])) if n in al else 0
    other = [Resource(k.s(n), quantity.value(q)) for n, q in al.items()
             if n not in ("cpu", "memory", "alpha.kubernetes.io/nvidia-gpu", "ephemeral-storage", "pods")]
    n_o, os_ = k.arr(Resource, other)
    av = [Avoid(0, None, None) if e is None else Avoid(1, k.s(e[0]), k.s(e[1])) for e in avoid_signatures(md.get("annotations"))]
    n_a, avs = k.arr(Avoid, av)
    imgs = [Image(*k.strs(img.get("names")), int(img.get("sizeBytes") or 0)) for img in st.get("images") or []]
    n_im, ims = k.arr(Image, imgs)
    return Node(k.s(md.get("name", "")), n_lab, labs, n_t, ts, int(bool(spec.get("unschedulable"))), n_c, cs,
                g("cpu", True), g("memory"), g("alpha.kubernetes.io/nvidia-gpu"), g("ephemeral-storage"), g("pods"),
                n_o, os_, n_a, avs, int(bool(st.get("images"))), n_im, ims)


def _pv_kind(spec):
    for key, kind, field in (("gcePersistentDisk", VOL_GCE_PD, "pdName"), ("awsElasticBlockStore", VOL_EBS, "volumeID"),
                             ("azureDisk", VOL_AZURE_DISK, "diskName")):
        if spec.get(key) is not None:
            return kind, spec[key].get(field, "")
    return VOL_OTHER, ""


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = abi.lib()
        P = C.c_void_p
        sigs = {"ksim_k8s_create": [C.POINTER(Options), C.POINTER(P)], "ksim_k8s_destroy": [P],
                "ksim_k8s_last_error": [P], "ksim_k8s_add_node": [P, C.POINTER(Node)], "ksim_k8s_add_pv": [P, C.POINTER(PV)],
                "ksim_k8s_add_pvc": [P, C.POINTER(PVC)], "ksim_k8s_add_storage_class": [P, C.POINTER(StorageClass)],
                "ksim_k8s_add_running_pod": [P, C.POINTER(Pod)], "ksim_k8s_add_queued_pod": [P, C.POINTER(Pod)],
                "ksim_k8s_build": [P], "ksim_k8s_open": [P, C.POINTER(abi.Config), C.c_int64, C.POINTER(P)],
                "ksim_k8s_node_count": [P], "ksim_k8s_node_name": [P, C.c_int64], "ksim_k8s_queue_length": [P],
                "ksim_k8s_pods": [P, P, P, P, P, P], "ksim_k8s_tables": [P, P, P, P, P],
                "ksim_k8s_describe": [P, P, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(C.c_int32),
                                      C.c_void_p, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int64)],
                "ksim_k8s_bind": [P, C.c_int64, C.c_int64],
                "ksim_k8s_open_ex": [P, C.POINTER(abi.Config), C.POINTER(Weights), C.POINTER(P)],
                "ksim_k8s_open_policy": [P, C.POINTER(abi.Config), C.POINTER(Weights), C.POINTER(PolicyArgs), C.POINTER(P)],
                "ksim_k8s_cache_create": [C.POINTER(CacheOptions), C.POINTER(P)], "ksim_k8s_cache_destroy": [P],
                "ksim_k8s_cache_last_error": [P], "ksim_k8s_cache_add_pv": [P, C.POINTER(PV)],
                "ksim_k8s_cache_add_pvc": [P, C.POINTER(PVC)],
                "ksim_k8s_cache_add_storage_class": [P, C.POINTER(StorageClass)],
                "ksim_k8s_cache_add_node": [P, C.POINTER(Node)],
                "ksim_k8s_cache_update_node": [P, C.POINTER(Node), C.POINTER(Node)],
                "ksim_k8s_cache_remove_node": [P, C.POINTER(Node)],
                "ksim_k8s_cache_assume_pod": [P, C.POINTER(Pod)], "ksim_k8s_cache_forget_pod": [P, C.POINTER(Pod)],
                "ksim_k8s_cache_add_pod": [P, C.POINTER(Pod)],
                "ksim_k8s_cache_update_pod": [P, C.POINTER(Pod), C.POINTER(Pod)],
                "ksim_k8s_cache_remove_pod": [P, C.POINTER(Pod)],
                "ksim_k8s_cache_schedule": [P, C.POINTER(Pod), C.c_int32, C.POINTER(abi.Result)],
                "ksim_k8s_cache_fit_error": [P, C.POINTER(abi.Result), C.c_char_p, C.c_int32],
                "ksim_k8s_cache_node_count": [P], "ksim_k8s_cache_node_name": [P, C.c_int64],
                "ksim_k8s_cache_handle": [P], "ksim_k8s_cache_stats": [P, C.POINTER(C.c_int64)]}
        for name, args in sigs.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = C.c_int
        L.ksim_k8s_destroy.restype = None
        L.ksim_k8s_last_error.restype = C.c_char_p
        L.ksim_k8s_node_name.restype = C.c_char_p
        L.ksim_k8s_node_count.restype = C.c_int64
        L.ksim_k8s_queue_length.restype = C.c_int64
        L.ksim_k8s_cache_destroy.restype = None
        L.ksim_k8s_cache_last_error.restype = C.c_char_p
        L.ksim_k8s_cache_node_count.restype = C.c_int64
        L.ksim_k8s_cache_node_name.restype = C.c_char_p
        L.ksim_k8s_cache_handle.restype = C.c_void_p
        L.ksim_k8s_cache_fit_error.restype = C.c_int32
        _lib = L
    return _lib


class K8sCluster:
    """A snapshot built by the C++ front end from Kubernetes-shaped dicts (the same arguments as
    ingest.Cluster.from_objects)."""

    def __init__(self, nodes, running_pods=(), pods=(), hard_weight=10, pvs=(), pvcs=(), storage_classes=(),
                 max_vols=None, port_slots=None, vol_slots=None, spread=None, spread_services_only=False,
                 image_locality=None):
        L = lib()
        opt = Options(int(hard_weight), (C.c_int32 * 3)(*(max_vols or (0, 0, 0))),
                      -1 if port_slots is None else int(port_slots), -1 if vol_slots is None else int(vol_slots),
                      0 if image_locality is None else (1 if image_locality else -1))
        h = C.c_void_p()
        self._check(L.ksim_k8s_create(C.byref(opt), C.byref(h)), None)
        self.h = h
        for x in nodes:
            k = _Keep()
            self._check(L.ksim_k8s_add_node(h, C.byref(flatten_node(k, x))))
        for x in pvs:
            k = _Keep()
            kind, vid = _pv_kind(x.get("spec") or {})
            md = x.get("metadata") or {}
            n_l, labs = _kvs(k, md.get("labels"))
            pv = PV(k.s(md.get("name", "")), n_l, labs, kind, k.s(vid), int((x.get("spec") or {}).get("nodeAffinity") is not None))
            self._check(L.ksim_k8s_add_pv(h, C.byref(pv)))
        for x in pvcs:
            k = _Keep()
            md, sp = x.get("metadata") or {}, x.get("spec") or {}
            sc = sp.get("storageClassName")
            self._check(L.ksim_k8s_add_pvc(h, C.byref(PVC(k.s(md.get("namespace", "")), k.s(md.get("name", "")),
                                                         k.s(sp.get("volumeName", "")), k.s(sc) if sc is not None else None))))
        for x in storage_classes:
            k = _Keep()
            mode = x.get("volumeBindingMode")
            self._check(L.ksim_k8s_add_storage_class(h, C.byref(StorageClass(k.s((x.get("metadata") or {}).get("name", "")),
                                                                             k.s(mode) if mode is not None else None))))
        for p in running_pods:
            k = _Keep()
            self._check(L.ksim_k8s_add_running_pod(h, C.byref(flatten_pod(k, p))))
        for p in pods:
            k = _Keep()
            self._check(L.ksim_k8s_add_queued_pod(h, C.byref(flatten_pod(k, p, spread_raw(spread, p, spread_services_only)))))
        self._check(L.ksim_k8s_build(h))

    def _check(self, rc, h="self"):
        if rc:
            msg = lib().ksim_k8s_last_error(self.h if h == "self" else None) or b""
            err = abi.KsimUnsupported if rc == abi.E_UNSUPPORTED else abi.KsimError
            raise err(rc, msg.decode())

    def close(self):
        if getattr(self, "h", None):
            lib().ksim_k8s_destroy(self.h)
            self.h = None

    __del__ = close

    @property
    def names(self):
        L = lib()
        return [L.ksim_k8s_node_name(self.h, i).decode() for i in range(L.ksim_k8s_node_count(self.h))]

    def pods(self):
        """(descriptors as POD_DTYPE, port keys, scalar requests as SCALAR_DTYPE)."""
        L = lib()
        pp, kp, sp = C.c_void_p(), C.c_void_p(), C.c_void_p()
        nk, ns = C.c_int64(), C.c_int64()
        self._check(L.ksim_k8s_pods(self.h, C.byref(pp), C.byref(kp), C.byref(nk), C.byref(sp), C.byref(ns)))
        n = L.ksim_k8s_queue_length(self.h)
        pods = np.frombuffer((C.c_char * (n * abi.POD_DTYPE.itemsize)).from_address(pp.value), abi.POD_DTYPE).copy() if n else \
            np.zeros(0, abi.POD_DTYPE)
        ports = np.ctypeslib.as_array((C.c_uint64 * nk.value).from_address(kp.value)).copy() if nk.value else np.zeros(0, np.uint64)
        sc = np.frombuffer((C.c_char * (ns.value * abi.SCALAR_DTYPE.itemsize)).from_address(sp.value), abi.SCALAR_DTYPE).copy() \
            if ns.value else np.zeros(0, abi.SCALAR_DTYPE)
        return pods, ports, sc

    def tables(self):
        """(NodeTable, ClassTables, AffinityTables, VolumeTables) structs viewing the library's arrays."""
        t = (abi.NodeTable(), abi.ClassTables(), abi.AffinityTables(), abi.VolumeTables())
        self._check(lib().ksim_k8s_tables(self.h, *[C.byref(x) for x in t]))
        return t

    def open_ex(self, cfg, prefer_avoid_weight=0, image_locality_weight=0):
        """ksim_k8s_open_ex: a policy that may weigh ImageLocalityPriority."""
        hh = C.c_void_p()
        w = Weights(int(prefer_avoid_weight), int(image_locality_weight))
        self._check(lib().ksim_k8s_open_ex(self.h, C.byref(cfg), C.byref(w), C.byref(hh)))
        return abi.Handle.adopt(hh, cfg)

    def open_policy(self, cfg, prefer_avoid_weight=0, image_locality_weight=0, label_presence=None,
                    service_affinity=None, label_priorities=(), services_select_pods=False):
        """ksim_k8s_open_policy: label_presence = (labels, presence) of CheckNodeLabelPresence,
        service_affinity = CheckServiceAffinity's labels, label_priorities = [(label, presence, weight,
        is_service_anti_affinity)] — a Policy's arguments (policy.key_sets / priority_arguments)."""
        hh = C.c_void_p()
        w = Weights(int(prefer_avoid_weight), int(image_locality_weight))
        keep = []
        a = policy_args(keep, label_presence, service_affinity, label_priorities, services_select_pods)
        self._check(lib().ksim_k8s_open_policy(self.h, C.byref(cfg), C.byref(w), C.byref(a), C.byref(hh)))
        return abi.Handle.adopt(hh, cfg)

    def open(self, cfg, prefer_avoid_weight=0):
        """A ksim_handle with everything loaded (abi.Handle-compatible wrapper)."""
        hh = C.c_void_p()
        self._check(lib().ksim_k8s_open(self.h, C.byref(cfg), int(prefer_avoid_weight), C.byref(hh)))
        return abi.Handle.adopt(hh, cfg)


def _pv_struct(k, x):
    kind, vid = _pv_kind(x.get("spec") or {})
    md = x.get("metadata") or {}
    n_l, labs = _kvs(k, md.get("labels"))
    return PV(k.s(md.get("name", "")), n_l, labs, kind, k.s(vid), int((x.get("spec") or {}).get("nodeAffinity") is not None))


def _pvc_struct(k, x):
    md, sp = x.get("metadata") or {}, x.get("spec") or {}
    sc = sp.get("storageClassName")
    return PVC(k.s(md.get("namespace", "")), k.s(md.get("name", "")), k.s(sp.get("volumeName", "")),
               k.s(sc) if sc is not None else None)


class K8sCache:
    """The C++ scheduler cache (ksim_k8s_cache_*): the per-pod drop-in a cgo adapter drives, with the
    method surface of ksim.cache.SchedulerCache / the reference's schedulercache.Cache (add_node,
    update_node, remove_node, assume_pod, forget_pod, add_pod, update_pod, remove_pod, schedule,
    schedule_one).  Objects are flattened exactly as a Go adapter would flatten v1 objects; every
    scheduling rule runs in the library.  Errors: KeyError with cache.go's message for cache-state
    errors (as SchedulerCache raises), KsimUnsupported / NoNodesAvailable / KsimError otherwise."""

    def __init__(self, predicates, priorities, device=0, mode=abi.MODE_AUTO, last_node_index=0, port_slots=8,
                 pvs=(), pvcs=(), storage_classes=(), hard_weight=10, spread=None, max_vols=None, label_presence=None,
                 service_affinity=None, custom_priorities=None):
        """label_presence / service_affinity / custom_priorities: a Policy's arguments (policy.key_sets,
        service_affinity_labels, priority_arguments) — evaluated in the library (ksim_k8s_policy_args)."""
        from . import scheduler
        self.predicates = list(predicates)
        self.prioritizers = list(priorities)
        self.spread = spread if spread else None
        names = {n for n, _ in priorities}
        custom = dict(custom_priorities or {})
        self._services_only = "ServiceSpreadingPriority" in names and "SelectorSpreadPriority" not in names
        # the reference fails on CheckNodeLabelPresence without its labelsPresence argument (as plan()
        # refuses it); with an empty labels list the predicate passes every node and is dropped
        if "CheckNodeLabelPresence" in self.predicates and label_presence is None:
            raise abi.KsimUnsupported(abi.E_UNSUPPORTED, "CheckNodeLabelPresence needs its labelsPresence argument")
        cfg = scheduler.make_config([k for k in predicates if k != "CheckNodeLabelPresence" or label_presence[0]],
                                    [(n, x) for n, x in priorities if n not in custom], device, mode, True,
                                    last_node_index, spread=self.spread is not None, configured=list(priorities))
        w = lambda key: sum(int(x) for n, x in priorities if n == key)
        self._keep_policy = []
        pol = None
        if label_presence is not None or service_affinity is not None or custom:
            weights = dict(priorities)
            pol = policy_args(self._keep_policy, label_presence, service_affinity,
                              [(a[1], a[2] if a[0] == "labelPreference" else True, int(weights[n]), a[0] == "serviceAntiAffinity")
                               for n, a in custom.items() if n in weights],
                              services_select_pods=bool(self.spread and self.spread.services))
        opt = CacheOptions(cfg, Weights(w("NodePreferAvoidPodsPriority"), w("ImageLocalityPriority")), int(hard_weight),
                           (C.c_int32 * 3)(*(max_vols or (0, 0, 0))), int(port_slots),
                           int("CheckVolumeBinding" in self.predicates), 0,
                           C.pointer(pol) if pol is not None else None)
        L = lib()
        h = C.c_void_p()
        rc = L.ksim_k8s_cache_create(C.byref(opt), C.byref(h))
        if rc:
            self.h = None
            raise self._err(rc, L.ksim_k8s_cache_last_error(None))
        self.h = h
        for x in pvs:
            k = _Keep()
            self._call("ksim_k8s_cache_add_pv", C.byref(_pv_struct(k, x)))
        for x in pvcs:
            k = _Keep()
            self._call("ksim_k8s_cache_add_pvc", C.byref(_pvc_struct(k, x)))
        for x in storage_classes:
            k = _Keep()
            mode_ = x.get("volumeBindingMode")
            sc = StorageClass(k.s((x.get("metadata") or {}).get("name", "")), k.s(mode_) if mode_ is not None else None)
            self._call("ksim_k8s_cache_add_storage_class", C.byref(sc))

    @staticmethod
    def _err(rc, msg):
        msg = (msg or b"").decode()
        if rc == abi.E_STATE:
            return KeyError(msg)
        if rc == abi.E_NO_NODES:
            return abi.NoNodesAvailable(rc, msg)
        return (abi.KsimUnsupported if rc == abi.E_UNSUPPORTED else abi.KsimError)(rc, msg)

    def _call(self, fn, *args):
        L = lib()
        rc = getattr(L, fn)(self.h, *args)
        if rc:
            raise self._err(rc, L.ksim_k8s_cache_last_error(self.h))

    def _pod(self, k, p):
        return C.byref(flatten_pod(k, p, spread_raw(self.spread, p, self._services_only)))

    def add_node(self, node):
        k = _Keep()
        self._call("ksim_k8s_cache_add_node", C.byref(flatten_node(k, node)))

    def update_node(self, old, new):
        k = _Keep()
        self._call("ksim_k8s_cache_update_node", C.byref(flatten_node(k, old)), C.byref(flatten_node(k, new)))

    def remove_node(self, node):
        k = _Keep()
        self._call("ksim_k8s_cache_remove_node", C.byref(flatten_node(k, node)))

    def assume_pod(self, pod):
        k = _Keep()
        self._call("ksim_k8s_cache_assume_pod", self._pod(k, pod))

    def forget_pod(self, pod):
        k = _Keep()
        self._call("ksim_k8s_cache_forget_pod", self._pod(k, pod))

    def add_pod(self, pod):
        k = _Keep()
        self._call("ksim_k8s_cache_add_pod", self._pod(k, pod))

    def update_pod(self, old, new):
        k = _Keep()
        self._call("ksim_k8s_cache_update_pod", self._pod(k, old), self._pod(k, new))

    def remove_pod(self, pod):
        k = _Keep()
        self._call("ksim_k8s_cache_remove_pod", self._pod(k, pod))

    def schedule(self, pod, assume=False):
        """genericScheduler.Schedule: the host name, or raises FitError (ksim.cache.FitError, message
        from the library) / abi.NoNodesAvailable; assume=True also runs Scheduler.assume."""
        from .cache import FitError
        k = _Keep()
        res = abi.Result()
        self._call("ksim_k8s_cache_schedule", self._pod(k, pod), abi.SCHEDULE_ASSUME if assume else abi.SCHEDULE_ONLY,
                   C.byref(res))
        self.last_fit_nodes = res.fit_nodes
        if res.node < 0:
            buf = C.create_string_buffer(4096)
            lib().ksim_k8s_cache_fit_error(self.h, C.byref(res), buf, 4096)
            import numpy as np
            err = FitError.__new__(FitError)  # the library's FitError text (scalar names are its own)
            Exception.__init__(err, buf.value.decode())
            err.num_nodes, err.hist = self.node_count(), np.asarray(list(res.reasons), np.int32)
            raise err
        return lib().ksim_k8s_cache_node_name(self.h, res.node).decode()

    def schedule_one(self, pod):
        from .cache import FitError
        try:
            return self.schedule(pod, assume=True), None
        except FitError as e:
            return None, str(e)

    @property
    def names(self):
        L = lib()
        return [L.ksim_k8s_cache_node_name(self.h, i).decode() for i in range(L.ksim_k8s_cache_node_count(self.h))]

    def node_count(self):
        return lib().ksim_k8s_cache_node_count(self.h)

    def _hcall(self, fn, *args):
        """A ksim_* call on the cache's own handle (borrowed: the cache destroys it)."""
        L = abi.lib()
        hh = C.c_void_p(lib().ksim_k8s_cache_handle(self.h))
        rc = getattr(L, fn)(hh, *args)
        if rc:
            raise abi.KsimError(rc, L.ksim_last_error(hh).decode(errors="replace"))

    @property
    def last_node_index(self):
        v = C.c_uint64()
        self._hcall("ksim_get_counter", C.byref(v))
        return v.value

    def stats(self):
        """(affinity loads, volume loads, volume grows, class loads)."""
        out = (C.c_int64 * 4)()
        self._call("ksim_k8s_cache_stats", out)
        return tuple(out)

    aff_reloads = property(lambda self: self.stats()[0])  # SchedulerCache's counters, same meaning
    vol_loads = property(lambda self: self.stats()[1])
    vol_grows = property(lambda self: self.stats()[2])

    def node_state(self):
        """Dynamic columns read back from the device, in name-rank order."""
        import numpy as np
        n = self.node_count()
        S = abi.MAX_SCALAR
        out = dict(req_cpu=np.zeros(n, np.int64), req_mem=np.zeros(n, np.int64), req_gpu=np.zeros(n, np.int64),
                   req_eph=np.zeros(n, np.int64), nz_cpu=np.zeros(n, np.int64), nz_mem=np.zeros(n, np.int64),
                   pod_count=np.zeros(n, np.int32), req_scalar=np.zeros((S, n), np.int64),
                   port_count=np.zeros(n, np.int32))
        st = abi.NodeState()
        for key, ct in (("req_cpu", C.c_int64), ("req_mem", C.c_int64), ("req_gpu", C.c_int64), ("req_eph", C.c_int64),
                        ("nz_cpu", C.c_int64), ("nz_mem", C.c_int64), ("pod_count", C.c_int32),
                        ("req_scalar", C.c_int64), ("port_count", C.c_int32)):
            setattr(st, key, abi.ptr(out[key], ct))
        self._hcall("ksim_read_nodes", C.byref(st))
        return out

    def close(self):
        if getattr(self, "h", None):
            lib().ksim_k8s_cache_destroy(self.h)
            self.h = None

    __del__ = close
