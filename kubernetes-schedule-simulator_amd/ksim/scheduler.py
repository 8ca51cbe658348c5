"""Host-side mirror of the reference's ScheduleAlgorithm plugin surface and simulator loop.

- Predicate / priority key sets and weights, exactly as the algorithm providers register
  them (vendor/k8s.io/kubernetes/pkg/scheduler/algorithmprovider/defaults/defaults.go:
  113-259, the TalkintDataProvider added at :36,214-216) or as a Policy lists them.
  Every supported key maps to a kernel feature bit or weight slot; any other key raises
  Unsupported (never a silently different result).
- GenericScheduler: the batch form of genericScheduler.Schedule + Scheduler.assume over a
  device-resident cluster (core/generic_scheduler.go:112-198, scheduler.go:366).
- FitError: message format of core/generic_scheduler.go:72-90.
- ClusterCapacity: the simulator's loop (pkg/scheduler/simulator.go:108-223): pods are
  popped LIFO from the expanded pod list (pkg/framework/store/store.go:223-233), each is
  scheduled and committed before the next; unschedulable pods are recorded and the run
  continues until the queue is empty.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import abi
from .ingest import Cluster, Unsupported, class_tables_struct

# predicates.go:129-138 keys → kernel bits
PREDICATE_BITS = {
    "CheckNodeCondition": abi.P_CHECK_NODE_CONDITION,
    "CheckNodeUnschedulable": abi.P_CHECK_NODE_UNSCHEDULABLE,
    "GeneralPredicates": abi.P_GENERAL,
    "HostName": abi.P_HOSTNAME,
    "PodFitsHostPorts": abi.P_HOST_PORTS,
    "MatchNodeSelector": abi.P_NODE_SELECTOR,
    "PodFitsResources": abi.P_RESOURCES,
    "PodToleratesNodeTaints": abi.P_TAINTS,
    "PodToleratesNodeNoExecuteTaints": abi.P_NOEXEC_TAINTS,
    "CheckNodeMemoryPressure": abi.P_MEM_PRESSURE,
    "CheckNodeDiskPressure": abi.P_DISK_PRESSURE,
    "CheckNodeLabelPresence": abi.P_LABEL_PRESENCE,   # with a Policy labelsPresence argument
    "MatchInterPodAffinity": abi.P_INTERPOD_AFFINITY,  # over the cluster's affinity tables
    "NoDiskConflict": abi.P_DISK_CONFLICT,              # over the cluster's volume tables
    "MaxEBSVolumeCount": abi.P_MAX_EBS,
    "MaxGCEPDVolumeCount": abi.P_MAX_GCE_PD,
    "MaxAzureDiskVolumeCount": abi.P_MAX_AZURE_DISK,
    "NoVolumeZoneConflict": abi.P_VOLUME_ZONE,
    "CheckServiceAffinity": abi.P_SERVICE_AFFINITY,     # with a Policy serviceAffinity argument
}
VOLUME_PREDICATE_BITS = abi.P_DISK_CONFLICT | abi.P_MAX_EBS | abi.P_MAX_GCE_PD | abi.P_MAX_AZURE_DISK | abi.P_VOLUME_ZONE
# factory/plugins.go:401-406 + defaults.go:165: part of every predicate map
MANDATORY_PREDICATES = ("CheckNodeCondition",)
# keys that are true for every pod the scheduler accepts: CheckVolumeBinding (PVCs only when
# bound to a PV without node affinity, ksim/volumes.py); "PodFitsPorts" is registered but absent
# from predicatesOrdering, so it never runs
TRIVIAL_PREDICATES = {"CheckVolumeBinding", "PodFitsPorts"}

PRIORITY_SLOTS = {"LeastRequestedPriority": abi.W_LEAST, "MostRequestedPriority": abi.W_MOST,
                  "BalancedResourceAllocation": abi.W_BALANCED, "TaintTolerationPriority": abi.W_TAINT_TOL,
                  "NodeAffinityPriority": abi.W_NODE_AFF, "InterPodAffinityPriority": abi.W_INTERPOD}
SPREAD_PRIORITIES = ("SelectorSpreadPriority", "ServiceSpreadingPriority")
# value on every node under supported inputs (no services/controllers in the simulator's store —
# with SpreadListers the spread priorities take the W_SPREAD slot —, no RC/RS-owned pods next to
# preferAvoidPods annotations)
CONST_PRIORITIES = {"SelectorSpreadPriority": 10, "ServiceSpreadingPriority": 10, "NodePreferAvoidPodsPriority": 10,
                    "EqualPriority": 1,
                    # image_locality.go:39-69: 0 on every node when no node lists status.images
                    "ImageLocalityPriority": 0}

DEFAULT_PREDICATES = ("NoVolumeZoneConflict", "MaxEBSVolumeCount", "MaxGCEPDVolumeCount", "MaxAzureDiskVolumeCount",
                      "MatchInterPodAffinity", "NoDiskConflict", "GeneralPredicates", "CheckNodeMemoryPressure",
                      "CheckNodeDiskPressure", "CheckNodeCondition", "PodToleratesNodeTaints", "CheckVolumeBinding")
DEFAULT_PRIORITIES = (("SelectorSpreadPriority", 1), ("InterPodAffinityPriority", 1), ("LeastRequestedPriority", 1),
                      ("BalancedResourceAllocation", 1), ("NodePreferAvoidPodsPriority", 10000),
                      ("NodeAffinityPriority", 1), ("TaintTolerationPriority", 1))
PROVIDERS = ("DefaultProvider", "ClusterAutoscalerProvider", "TalkintDataProvider")


def provider(name: str):
    """registerAlgorithmProvider (defaults.go:207-217)."""
    if name not in PROVIDERS:
        raise Unsupported("algorithm provider %r is not registered" % name)
    pri = list(DEFAULT_PRIORITIES)
    if name != "DefaultProvider":  # copyAndReplace(LeastRequested → MostRequested)
        pri = [("MostRequestedPriority", w) if n == "LeastRequestedPriority" else (n, w) for n, w in pri]
    return list(DEFAULT_PREDICATES), pri


def make_config(predicates, priorities, device=0, mode=abi.MODE_AUTO, collect_reasons=True, last_node_index=0,
                spread=False, configured=None):
    """spread: the cluster has SelectorSpread selectors (Cluster.spread_active): the spread priority
    scores per node (KSIM_W_SELECTOR_SPREAD) instead of being the constant MaxPriority.
    configured: the whole prioritizer list when `priorities` leaves some out (Policy priorities
    with arguments, the auxiliary priority): only an empty one means EqualPriorityMap."""
    cfg = abi.Config()
    cfg.device = device
    cfg.mode = mode
    bits = 0
    for k in list(predicates) + list(MANDATORY_PREDICATES):
        if k in PREDICATE_BITS:
            bits |= PREDICATE_BITS[k]
        elif k not in TRIVIAL_PREDICATES:
            raise Unsupported("predicate %r is outside the supported key set" % k)
    cfg.predicates = bits
    const = 0
    seen = set()
    for name, w in priorities:
        if name in seen:
            raise abi.KsimError(abi.E_INVAL, "duplicate priority %r" % name)
        seen.add(name)
        if w <= 0:
            raise abi.KsimError(abi.E_INVAL, "priority %r: weight must be positive" % name)
        if name in PRIORITY_SLOTS:
            cfg.weights[PRIORITY_SLOTS[name]] = w
        elif spread and name in SPREAD_PRIORITIES:
            if cfg.weights[abi.W_SPREAD]:
                raise Unsupported("SelectorSpreadPriority and ServiceSpreadingPriority together with spread selectors")
            cfg.weights[abi.W_SPREAD] = w
        elif name in CONST_PRIORITIES:
            const += CONST_PRIORITIES[name] * w
        else:
            raise Unsupported("priority %r is outside the supported key set" % name)
    empty = not (priorities if configured is None else configured)
    cfg.no_priorities = 1 if empty else 0
    if empty:
        const = 1
    cfg.const_score = const
    cfg.collect_reasons = 1 if collect_reasons else 0
    cfg.last_node_index = last_node_index
    return cfg


REASON_TEXT = {
    abi.R_NOT_READY: "node(s) were not ready",
    abi.R_OUT_OF_DISK: "node(s) were out of disk space",
    abi.R_NET_UNAVAIL: "node(s) had unavailable network",
    abi.R_UNSCHEDULABLE: "node(s) were unschedulable",
    abi.R_PODS: "Insufficient pods",
    abi.R_CPU: "Insufficient cpu",
    abi.R_MEMORY: "Insufficient memory",
    abi.R_GPU: "Insufficient alpha.kubernetes.io/nvidia-gpu",
    abi.R_EPHEMERAL: "Insufficient ephemeral-storage",
    abi.R_HOSTNAME: "node(s) didn't match the requested hostname",
    abi.R_HOST_PORTS: "node(s) didn't have free ports for the requested pod ports",
    abi.R_NODE_SELECTOR: "node(s) didn't match node selector",
    abi.R_TAINTS: "node(s) had taints that the pod didn't tolerate",
    abi.R_MEM_PRESSURE: "node(s) had memory pressure",
    abi.R_DISK_PRESSURE: "node(s) had disk pressure",
    abi.R_LABEL_PRESENCE: "node(s) didn't have the requested labels",
    abi.R_POD_AFFINITY: "node(s) didn't match pod affinity/anti-affinity",
    abi.R_EXISTING_ANTI: "node(s) didn't satisfy existing pods anti-affinity rules",
    abi.R_AFFINITY_RULES: "node(s) didn't match pod affinity rules",
    abi.R_ANTI_AFFINITY_RULES: "node(s) didn't match pod anti-affinity rules",
    abi.R_DISK_CONFLICT: "node(s) had no available disk",
    abi.R_MAX_VOLUME_COUNT: "node(s) exceed max volume count",
    abi.R_VOLUME_ZONE: "node(s) had no available volume zone",
    abi.R_SERVICE_AFFINITY: "node(s) didn't match service affinity",
}


def reason_strings(mask: int, scalar_names=()):
    out = []
    for r in range(abi.NREASONS):
        if (mask >> r) & 1:
            out.append(reason_text(r, scalar_names))
    return out


def reason_text(r, scalar_names=()):
    if abi.R_SCALAR0 <= r < abi.R_SCALAR0 + abi.MAX_SCALAR:
        return "Insufficient " + scalar_names[r - abi.R_SCALAR0]
    return REASON_TEXT[r]


def fit_error_message(num_nodes, hist, scalar_names=()):
    """FitError.Error (core/generic_scheduler.go:72-90)."""
    parts = sorted("%d %s" % (int(v), reason_text(r, scalar_names)) for r, v in enumerate(hist) if v)
    return "0/%d nodes are available: %s." % (num_nodes, ", ".join(parts))


def label_set_priority(spec, label_set):
    """Map score of a Policy custom priority that is a function of the node's labels alone:
    NodeLabelPriority (priorities/node_label.go:42-58) and, with no services selecting the pod, the
    ServiceAntiAffinity priority (selector_spreading.go:221-275: no first service selector, so every
    count is 0 and a node scores MaxPriority when it has the label, 0 otherwise)."""
    if spec[0] == "labelPreference":
        return 10 if (spec[1] in label_set) == spec[2] else 0
    return 10 if spec[1] in label_set else 0


def class_tables_for(tables, priorities, label_sets=(), custom=None):
    """The class tables a scheduler with these priorities loads, and the weighted per-NodeAffinity-
    class addends (ksim_class_tables.na_add) or None.

    NodePreferAvoidPodsPriority (node_prefer_avoid_pods.go:32-68) and ImageLocalityPriority
    (image_locality.go:39-88) are functions of (pod class, label set) — the label set carries the
    node's preferAvoidPods annotation and its images, the class the pod's controller and container
    images — and the Policy's labelPreference / serviceAntiAffinity priorities
    (label_set_priority) of the label set alone.
    When the policy weighs them and they differ across the nodes some pod class sees, the
    NodeAffinity class dimension is re-keyed by (preferred weight, summed addend) — by the addend
    alone if NodeAffinityPriority is not configured — and each class adds its weighted score.
    Otherwise NodePreferAvoidPods is the constant MaxPriority x weight of const_score."""
    custom = custom or {}
    w_pa = sum(int(x) for n, x in priorities if n == "NodePreferAvoidPodsPriority")
    w_im = sum(int(x) for n, x in priorities if n == "ImageLocalityPriority")
    im_s = tables.get("im_s")
    im_on = bool(w_im and im_s is not None and im_s.any())
    w_custom = [(custom[n], int(x)) for n, x in priorities if n in custom]
    L = tables["na_class"].shape[1] if tables["na_class"].ndim == 2 else len(label_sets)
    lab_add = np.zeros(L, np.int64)
    for spec, w in w_custom:
        lab_add += np.array([w * label_set_priority(spec, ls) for ls in label_sets], np.int64)
    pa_on = bool(w_pa and tables.get("pa_split"))
    if not pa_on and not im_on and not lab_add.any():
        return tables, None
    use_w = any(n == "NodeAffinityPriority" for n, _ in priorities)
    d = dict(tables)
    Cn = d["n_classes"]
    nac = np.zeros_like(tables["na_class"])
    nna = np.ones(Cn, np.int32)
    avs = []
    for k in range(Cn):
        pa = [int(p) * w_pa if pa_on else 0 for p in tables["na_p"][k]]
        if im_on:
            pa = [a + w_im * int(x) for a, x in zip(pa, im_s[k])]
        keys = list(zip((int(x) if use_w else 0 for x in tables["na_w"][k]), (a + int(b) for a, b in zip(pa, lab_add))))
        av = sorted(set(keys))
        if int(tables["n_tt"][k]) * len(av) > abi.MAX_WIDE:
            raise Unsupported("pod class needs %d x %d reduce classes (> %d)" % (int(tables["n_tt"][k]), len(av), abi.MAX_WIDE))
        nna[k] = len(av)
        avs.append(av)
        pos = {x: i for i, x in enumerate(av)}
        nac[k, :] = [pos[x] for x in keys]
    # one row width for every value array: the class table's, or wider when the addends split more classes
    W = max([tables["tt_val"].shape[1]] + [len(av) for av in avs])
    nav = np.zeros((Cn, W), np.int64)
    add = np.zeros((Cn, W), np.int64)
    for k, av in enumerate(avs):
        nav[k, :len(av)] = [w for w, _ in av]
        add[k, :len(av)] = [p for _, p in av]
    ttv = np.zeros((Cn, W), np.int64)
    ttv[:, :tables["tt_val"].shape[1]] = tables["tt_val"]
    d.update(na_class=nac, n_na=nna, na_val=nav, tt_val=ttv, pa_in_add=pa_on)
    return d, add


def service_affinity_table(class_specs, label_sets, affinity_labels):
    """CheckServiceAffinity (predicates.go:980-1016) with no service selecting the pod: per pod
    class the label sets carrying the class's nodeSelector values of `affinity_labels`
    (FindLabelsInSet, CreateSelectorFromLabels — labels.Set.AsSelector, Everything when empty or
    invalid).  Returns ([n_classes][words] bits, per-class "fails somewhere")."""
    from . import labels as L
    C, S = len(class_specs), len(label_sets)
    words = max((S + 31) // 32, 1)
    ok = np.zeros((C, words), np.uint32)
    need = np.zeros(C, bool)
    for k, spec in enumerate(class_specs):
        sel = (spec or {}).get("nodeSelector") or {}
        al = {x: sel[x] for x in affinity_labels if x in sel}
        req = L.from_set(al)
        for j, ls in enumerate(label_sets):
            if L.matches(req, dict(ls)):
                ok[k, j >> 5] |= np.uint32(1 << (j & 31))
            else:
                need[k] = True
    return ok, need


def check_volume_support(cluster, predicates):
    """Refuse inputs on which a configured volume predicate returns an error instead of a verdict
    (ksim/volumes.py): findNodesThatFit then aborts the pod's cycle (core/generic_scheduler.go:351-353)
    and the simulator's requeue path takes over, which this batch form does not restate."""
    if cluster.volume_index is None:
        return
    errs = cluster.volume_index.errors
    keys = set(predicates)
    maxpd = keys & {"MaxEBSVolumeCount", "MaxGCEPDVolumeCount", "MaxAzureDiskVolumeCount"}
    if "claim_name" in errs and (maxpd or "NoVolumeZoneConflict" in keys):
        raise Unsupported("a PersistentVolumeClaim volume without a claim name (the volume predicates err)")
    if "binding" in errs and "CheckVolumeBinding" in keys:
        raise Unsupported("CheckVolumeBinding with a PVC that is not bound to a PV without node affinity "
                          "(FindPodVolumes errs or needs the volume binder)")
    if cluster.volumes is not None and cluster.volumes["zone_err"] and "NoVolumeZoneConflict" in keys:
        raise Unsupported("NoVolumeZoneConflict with a PVC the PV / PVC listers cannot resolve on a zone-labelled node")


def label_presence_flags(label_sets, label_set_ids, label_presence):
    """KSIM_N_LABEL_PRESENCE per node: CheckNodeLabelPresence (predicates.go:875-910) fails when
    a listed label's presence differs from `presence`; a function of the node's label set."""
    labels_, presence = label_presence
    bad = np.array([any((k in ls) != presence for k in labels_) for ls in label_sets], bool)
    return np.where(bad[np.asarray(label_set_ids)], abi.N_LABEL_PRESENCE, 0).astype(np.uint32)


@dataclass
class Plan:
    """What a scheduler over `cluster` loads, derived on the host alone (no device): the config,
    the node flags, the class tables with their NodePreferAvoidPods addends, the pod queue as
    loaded (affinity / volume / service-affinity fields adjusted to the configured keys), and the
    affinity / volume tables when a configured key reads them (else None)."""
    cfg: object
    flags: object          # node flags with the CheckNodeLabelPresence verdicts, or None (the cluster's)
    tables: dict
    na_add: object
    const_score: int
    pods: object
    affinity: object
    volumes: object
    use_zone: bool


def plan(cluster: Cluster, predicates, priorities, device=0, mode=abi.MODE_AUTO, collect_reasons=True,
         last_node_index=0, label_presence=None, custom_priorities=None, service_affinity=None) -> Plan:
    """The host half of GenericScheduler's construction (also what the table-level C oracle runs
    on): validates the key sets against the cluster's inputs (Unsupported where the reference errs
    or where this restatement stops) and builds every table the library loads."""
    predicates = list(predicates)
    prioritizers = list(priorities)
    custom_priorities = dict(custom_priorities or {})
    aux = getattr(cluster, "aux", None)
    aux_active = bool(getattr(cluster, "aux_active", False))
    aux_weight, aux_const = 0, 0
    saa = [(n, int(w)) for n, w in prioritizers if n in custom_priorities and custom_priorities[n][0] == "serviceAntiAffinity"]
    if saa and aux is not None and aux[0] == "service_anti_affinity" and aux_active:
        # ServiceAntiAffinity with services: the auxiliary counted priority (the pods' single
        # selecting service; Cluster.from_objects refused two or more)
        if len(saa) > 1 or custom_priorities[saa[0][0]][1] != aux[1]:
            raise Unsupported("serviceAntiAffinity priorities other than the one the cluster was built for (%r)" % (aux[1],))
        aux_weight = saa[0][1]
        prioritizers = [(n, w) for n, w in prioritizers if n != saa[0][0]]
        custom_priorities.pop(saa[0][0])
    elif saa and getattr(cluster, "spread_active", False) and not (aux is not None and aux[0] == "service_anti_affinity"):
        raise Unsupported("a serviceAntiAffinity priority with services selecting the pods needs the cluster built "
                          "with aux=('service_anti_affinity', label)")
    names = {n for n, _ in prioritizers}
    if aux is not None and aux[0] == "service_spreading" and {"SelectorSpreadPriority", "ServiceSpreadingPriority"} <= names:
        # ServiceSpreadingPriority next to SelectorSpreadPriority: the auxiliary counted priority over
        # the services-only selectors (MaxPriority everywhere, a constant, when none selects a pod)
        w = sum(int(x) for n, x in prioritizers if n == "ServiceSpreadingPriority")
        if aux_active:
            aux_weight = w
        else:
            aux_const = 10 * w
        prioritizers = [(n, x) for n, x in prioritizers if n != "ServiceSpreadingPriority"]
    if any(n == "NodeAffinityPriority" for n, _ in prioritizers) and cluster.bad_affinity_classes:
        raise Unsupported("NodeAffinityPriority: a preferred node-affinity term does not parse")
    if (any(n == "ImageLocalityPriority" for n, _ in prioritizers) and cluster.node_images
            and not getattr(cluster, "image_locality", False)):
        raise Unsupported("ImageLocalityPriority with nodes that list status.images, on a cluster built "
                          "without image interning (Cluster.from_objects(image_locality=True))")
    if "CheckNodeLabelPresence" in predicates and label_presence is None:
        raise Unsupported("CheckNodeLabelPresence needs its labelsPresence argument")
    svc_dyn = False
    if "CheckServiceAffinity" in predicates:
        if service_affinity is None:
            raise Unsupported("CheckServiceAffinity needs its serviceAffinity argument")
        if getattr(cluster, "svc_any", getattr(cluster, "spread_active", False)):
            # services select queued pods: the lender check needs the cluster built for these labels
            if getattr(cluster, "svc_labels", None) != list(service_affinity):
                raise Unsupported("CheckServiceAffinity with services selecting the pods needs the cluster built with "
                                  "service_affinity=%r" % (list(service_affinity),))
            svc_dyn = bool(cluster.svc_active)
    cfg = make_config([k for k in predicates if k != "CheckNodeLabelPresence" or label_presence],
                      [(n, w) for n, w in prioritizers if n not in custom_priorities],
                      device, mode, collect_reasons, last_node_index,
                      spread=bool(getattr(cluster, "spread_active", False)), configured=list(priorities))
    check_volume_support(cluster, predicates)
    flags = None
    if label_presence is not None and "CheckNodeLabelPresence" in predicates:
        fl = cluster.cols["flags"] | label_presence_flags(cluster.label_sets.items, cluster.cols["label_set"],
                                                            label_presence)
        flags = np.ascontiguousarray(fl, np.uint32)
    tables, na_add = class_tables_for(cluster.tables, prioritizers, cluster.label_sets.items, custom_priorities)
    # const_score without NodePreferAvoidPods when its per-class addends carry it
    const_score = cfg.const_score - (10 * sum(int(x) for n, x in prioritizers if n == "NodePreferAvoidPodsPriority")
                                     if tables.get("pa_in_add") else 0) + aux_const
    pods = np.ascontiguousarray(cluster.pods)
    if "CheckServiceAffinity" in predicates:
        ok, need = service_affinity_table(cluster.classes.items or [{}], cluster.label_sets.items, service_affinity)
        tables = dict(tables, svc_ok=ok)
        if len(pods):
            pods = pods.copy()
            pods["flags"] |= np.where(need[pods["cls"]], abi.POD_NEED_SVC_AFFINITY, 0).astype(np.uint32)
    affinity = None
    if cluster.affinity is not None:
        if cfg.predicates & abi.P_INTERPOD_AFFINITY or svc_dyn or \
                ((cfg.weights[abi.W_INTERPOD] or cfg.weights[abi.W_SPREAD] or aux_weight) and not cfg.no_priorities):
            affinity = cluster.affinity
            if cluster.affinity.get("aux_pair") is not None or cluster.affinity.get("svc_on"):
                affinity = dict(cluster.affinity, aux_weight=aux_weight, svc_use=svc_dyn)
        elif len(pods):  # neither MatchInterPodAffinity nor its priority: the terms change nothing
            pods = pods.copy()
            pods["aff_ident"] = 0
            pods["aff_class"] = 0
    volumes = None
    if cluster.volumes is not None:
        if cfg.predicates & VOLUME_PREDICATE_BITS:
            volumes = cluster.volumes
        elif len(pods):  # no volume predicate: the pods' volumes change nothing
            pods = pods.copy()
            pods["vol_class"] = 0
    return Plan(cfg, flags, tables, na_add, const_score, pods, affinity, volumes, "NoVolumeZoneConflict" in predicates)


class GenericScheduler:
    """Batch drop-in for genericScheduler + Scheduler.assume on one MI355X.  label_presence:
    (labels, presence) of a Policy's CheckNodeLabelPresence predicate (policy.key_sets)."""

    def __init__(self, cluster: Cluster, predicates, priorities, device=0, mode=abi.MODE_AUTO,
                 collect_reasons=True, last_node_index=0, label_presence=None, custom_priorities=None,
                 service_affinity=None):
        self.cluster = cluster
        self.predicates = list(predicates)
        self.prioritizers = list(priorities)
        # Policy priorities registered with a labelPreference / serviceAntiAffinity argument, by name
        self.custom_priorities = dict(custom_priorities or {})
        p = self.plan = plan(cluster, predicates, priorities, device, mode, collect_reasons, last_node_index,
                             label_presence, custom_priorities, service_affinity)
        self.cfg = p.cfg
        self.h = abi.Handle(self.cfg)
        table = cluster.node_table()
        if p.flags is not None:
            self._flags = p.flags
            table.flags = abi.ptr(self._flags, C.c_uint32)
        self.h.call("ksim_load_nodes", C.byref(table))
        self.tables, self.na_add, self.const_score = p.tables, p.na_add, p.const_score
        self.h.call("ksim_load_classes", C.byref(class_tables_struct(self.tables, self.na_add)))
        self.affinity = p.affinity
        if self.affinity is not None:
            from .affinity import tables_struct
            self.h.call("ksim_load_affinity", C.byref(tables_struct(self.affinity)))
        self.volumes = p.volumes
        if self.volumes is not None:
            from .volumes import tables_struct as vol_struct
            self.h.call("ksim_load_volumes", C.byref(vol_struct(self.volumes, p.use_zone)))
        pods = self._pods = p.pods
        self.h.call("ksim_load_pods", abi.vptr(pods), len(pods), abi.vptr(cluster.pod_ports), len(cluster.pod_ports),
                    abi.vptr(cluster.pod_scalars), len(cluster.pod_scalars))
        self.last_stats = None

    def volume_state(self):
        """The device's volume slots ([vol_slots][n]) and per-node slot counts."""
        d = self.volumes
        slots = np.zeros_like(d["slots"])
        cnt = np.zeros_like(d["slot_count"])
        self.h.call("ksim_read_volumes", abi.vptr(slots), abi.vptr(cnt))
        return slots, cnt

    def schedule(self, first=0, count=None):
        """Schedule + assume pods [first, first+count) in order.
        Returns (node index per pod (-1 = FitError), reason histograms or None, stats)."""
        n = len(self._pods)
        count = n - first if count is None else count
        out = np.zeros(count, np.int32)
        reasons = np.zeros((count, abi.NREASONS), np.int32) if self.cfg.collect_reasons else None
        st = abi.Stats()
        self.h.call("ksim_schedule", first, count, abi.vptr(out), abi.vptr(reasons), C.byref(st))
        self.last_stats = st
        return out, reasons, st

    def sweep(self, scenarios, first=0, count=None):
        """Capacity-planning what-if (ksim_sweep): every scenario — a prioritizer list of map
        priorities, e.g. [("LeastRequestedPriority", 3), ("BalancedResourceAllocation", 1)] —
        schedules pods [first, first+count) on its own copy of the current node state, from the
        current lastNodeIndex, with this scheduler's predicates.  The scheduler's own state is
        unchanged.  Returns (placements [n_scen][count], final counters [n_scen], stats)."""
        n = len(self._pods)
        count = n - first if count is None else count
        w = np.zeros((len(scenarios), abi.NW), np.int64)
        for k, pri in enumerate(scenarios):
            cfg = make_config(self.predicates, pri)
            if cfg.no_priorities != self.cfg.no_priorities:
                raise Unsupported("a sweep scenario needs a non-empty prioritizer list like the scheduler's")
            w[k] = list(cfg.weights)
        out = np.zeros((len(scenarios), count), np.int32)
        ctr = np.zeros(len(scenarios), np.uint64)
        st = abi.Stats()
        self.h.call("ksim_sweep", abi.vptr(w), len(scenarios), first, count, abi.vptr(out), abi.vptr(ctr), C.byref(st))
        self.last_stats = st
        return out, ctr, st

    def evaluate(self, pod):
        """Per-node (fit, reason mask, map score, reduce class) for one loaded pod (no commit)."""
        n = self.cluster.n_nodes
        fit = np.zeros(n, np.uint8)
        rs = np.zeros(n, np.uint32)
        sc = np.zeros(n, np.int64)
        rc = np.zeros(n, np.uint8)
        self.h.call("ksim_evaluate", pod, abi.vptr(fit), abi.vptr(rs), abi.vptr(sc), abi.vptr(rc))
        return fit.astype(bool), rs, sc, rc

    def priority_scores(self, pod, over=None):
        """Total priority score per node as PrioritizeNodes reports it (map + reduce + the
        constant priorities) over the node subset `over` (default: fit nodes)."""
        fit, _, sc, rc = self.evaluate(pod)
        idx = np.nonzero(fit)[0] if over is None else np.asarray(over)
        p = self.cluster.pods[pod]
        t = self.tables
        cls = int(p["cls"])
        use_na = bool(self.cfg.weights[abi.W_NODE_AFF]) or self.na_add is not None
        k2 = int(t["n_na"][cls]) if use_na else 1
        tv = t["tt_val"][cls][rc[idx] // k2]
        av = t["na_val"][cls][rc[idx] % k2]
        total = sc[idx].copy()
        if self.cfg.weights[abi.W_TAINT_TOL]:
            total += self.cfg.weights[abi.W_TAINT_TOL] * _normalize(tv, True)
        if self.cfg.weights[abi.W_NODE_AFF]:
            total += self.cfg.weights[abi.W_NODE_AFF] * _normalize(av, False)
        if self.na_add is not None:
            total += self.na_add[cls][rc[idx] % k2]
        return idx, total + self.const_score

    def node_state(self):
        n = self.cluster.n_nodes
        S = self.cluster.cols["alloc_scalar"].shape[0]
        P = self.cluster.port_slots
        out = dict(req_cpu=np.zeros(n, np.int64), req_mem=np.zeros(n, np.int64), req_gpu=np.zeros(n, np.int64),
                   req_eph=np.zeros(n, np.int64), nz_cpu=np.zeros(n, np.int64), nz_mem=np.zeros(n, np.int64),
                   pod_count=np.zeros(n, np.int32), req_scalar=np.zeros((S, n), np.int64),
                   ports=np.zeros((P, n), np.uint64), port_count=np.zeros(n, np.int32))
        st = abi.NodeState()
        for k, ct in (("req_cpu", C.c_int64), ("req_mem", C.c_int64), ("req_gpu", C.c_int64), ("req_eph", C.c_int64),
                      ("nz_cpu", C.c_int64), ("nz_mem", C.c_int64), ("pod_count", C.c_int32),
                      ("req_scalar", C.c_int64), ("ports", C.c_uint64), ("port_count", C.c_int32)):
            setattr(st, k, abi.ptr(out[k], ct))
        self.h.call("ksim_read_nodes", C.byref(st))
        return out

    @property
    def last_node_index(self):
        v = C.c_uint64()
        self.h.call("ksim_get_counter", C.byref(v))
        return v.value

    def close(self):
        self.h.close()


class ShardedScheduler(GenericScheduler):
    """Rank `rank` of a node-sharded scheduler: loads the contiguous
    name-rank shard [rank*n/world, (rank+1)*n/world) of `cluster` and the whole pod queue;
    all ranks call schedule() with the same ranges.  Connect the ranks first: connect_local
    (ranks driven from this process) or export_handle / connect (one process per device)."""

    def __init__(self, cluster: Cluster, predicates, priorities, rank, world, device=0, collect_reasons=False,
                 last_node_index=0, custom_priorities=None):
        """collect_reasons: each rank's schedule() returns, for every pod no node of the world fits,
        the reason histogram of its own shard; merge_sharded_reasons sums the ranks' into the
        FitError histogram over every node (generic_scheduler.go:51-90 builds FitError from the
        failedPredicateMap of all nodes, :289-378, and every node lies in exactly one shard)."""
        n = cluster.n_nodes
        self.lo, self.hi = rank * n // world, (rank + 1) * n // world
        self.rank, self.world = rank, world
        super().__init__(cluster.shard(self.lo, self.hi), predicates, priorities, device=device,
                         mode=abi.MODE_PERSISTENT, collect_reasons=collect_reasons, last_node_index=last_node_index,
                         custom_priorities=custom_priorities)
        self.full_cluster = cluster
        self.h.call("ksim_shard_setup", rank, world, self.lo)

    def export_handle(self) -> bytes:
        buf = (C.c_uint8 * abi.IPC_HANDLE_BYTES)()
        self.h.call("ksim_shard_export", buf)
        return bytes(buf)

    def connect(self, peer, handle: bytes):
        buf = (C.c_uint8 * abi.IPC_HANDLE_BYTES).from_buffer_copy(handle)
        self.h.call("ksim_shard_connect", peer, buf)

    def connect_local(self, peer, other: "ShardedScheduler"):
        self.h.call("ksim_shard_connect_local", peer, other.h.h)

    def connect_torch(self, dist):
        """Exchange IPC handles with every rank of an initialised torch.distributed group."""
        hs = [None] * self.world
        dist.all_gather_object(hs, self.export_handle())
        for r, hb in enumerate(hs):
            if r != self.rank:
                self.connect(r, hb)


def connect_local_world(scheds):
    """Connect the ranks of a node-sharded scheduler driven from this process."""
    for s in scheds:
        for t in scheds:
            if s is not t:
                s.connect_local(t.rank, t)


def merge_sharded(outs):
    """Per-rank ksim_schedule outputs (-2 = another rank's node) → global placements."""
    return np.max(np.stack(outs), axis=0)


def merge_sharded_reasons(reasons):
    """Per-rank FitError histograms ([pods][KSIM_NREASONS], each over its own shard) → the
    histogram over every node: their sum.  Host-side, once per call (a torch.distributed
    all_reduce(SUM) of the same arrays between processes)."""
    return np.sum(np.stack([np.asarray(r, np.int64) for r in reasons]), axis=0).astype(np.int32)


def _normalize(vals, reverse):
    """NormalizeReduce over a value vector (priorities/reduce.go:29-64)."""
    vals = np.asarray(vals, np.int64)
    mx = int(vals.max()) if len(vals) else 0
    if mx == 0:
        return np.full(len(vals), 10, np.int64) if reverse else vals.copy()
    s = (10 * vals) // mx
    return 10 - s if reverse else s


# ----------------------------------------------------------------------------- simulator
def expand_simulation_pods(spec_list, namespace="", uid=None):
    """ParseSimulationPod (cmd/app/options/options.go:73-99): each SimulationPod's pod deep-copied
    `num` times with UID = name = a fresh uuid, labels replaced by {SimulationName: name} and the
    namespace set.  uid: None → deterministic "<SimulationName>-<i>" (so runs are reproducible);
    "uuid" → uuid4 strings as the reference makes them; or a callable (sp name, i) → str."""
    import copy
    import uuid as _uuid
    out = []
    for sp in spec_list:
        for i in range(int(sp.get("num", 0))):
            if uid is None:
                u = "%s-%d" % (sp["name"], i)
            elif uid == "uuid":
                u = str(_uuid.uuid4())
            else:
                u = uid(sp["name"], i)
            pod = copy.deepcopy(sp.get("pod") or {})
            meta = pod.setdefault("metadata", {})
            meta.update({"uid": u, "name": u, "namespace": namespace, "labels": {"SimulationName": sp["name"]}})
            pod.setdefault("spec", {})
            out.append(pod)
    return out


def load_podspec(path):
    """The --podspec file: a YAML or JSON list of SimulationPod{name, num, pod}
    (pkg/api/api.go:79-83, cmd/app/options/options.go:73-99)."""
    import yaml
    with open(path) as f:
        return yaml.safe_load(f)


def load_checkpoint(nodes_path, pods_path=None):
    """The offline snapshot (pkg/main.go:147-179 getNodeCheckPoint / getPodsCheckPoint): JSON
    arrays of v1.Node and v1.Pod.  Returns (nodes, pods)."""
    import json
    with open(nodes_path) as f:
        nodes = json.load(f)
    pods = []
    if pods_path:
        with open(pods_path) as f:
            pods = json.load(f)
    if not isinstance(nodes, list) or not isinstance(pods, list):
        raise abi.KsimError(abi.E_INVAL, "checkpoint files must hold JSON arrays of v1.Node / v1.Pod")
    return nodes, pods


@dataclass
class Report:
    """The simulation's outcome: (pod, node) in bind order, (pod, FitError text) for failed pods,
    the framework.Status the reference reports from (report.status, pod objects as the
    simulator leaves them) and GetReport's review (report.review)."""
    successful: list = field(default_factory=list)   # (pod name, node name) in bind order
    failed: list = field(default_factory=list)       # (pod name, FitError message)
    stop_reason: str = ""
    stats: object = None
    last_node_index: int = 0
    status: object = None
    review: object = None

    def text(self) -> str:
        """ClusterCapacityReviewPrint's output."""
        from .report import review_text
        return review_text(self.review)


class ClusterCapacity:
    """The simulator (pkg/scheduler/simulator.go:286-342 New, :187-213 Run): nodes and running
    pods of a snapshot, the simulation pods popped LIFO from the expanded podspec list
    (pkg/framework/store/store.go:223-233), each scheduled and committed before the next; a
    provider name, explicit key lists or a Policy (policy.key_sets) configure the algorithm."""

    def __init__(self, nodes, running_pods, simulation_pods, provider_name="DefaultProvider",
                 predicates=None, priorities=None, device=0, mode=abi.MODE_AUTO, collect_reasons=True,
                 policy_obj=None, pvs=(), pvcs=(), storage_classes=(), spread=None):
        label_presence = None
        custom = None
        svc_aff = None
        if policy_obj is not None:
            from .policy import key_sets, priority_arguments, service_affinity_labels
            predicates, priorities, label_presence = key_sets(policy_obj)
            custom = priority_arguments(policy_obj)
            svc_aff = service_affinity_labels(policy_obj)
        if predicates is None or priorities is None:
            p, q = provider(provider_name)
            predicates = p if predicates is None else predicates
            priorities = q if priorities is None else priorities
        self.order = list(reversed(simulation_pods))   # PodQueue.Pop takes the last element
        self.running = list(running_pods)
        # pvs / pvcs / storage_classes: the simulator's listers are empty; other callers may fill them
        names = {n for n, _ in priorities}
        both = {"SelectorSpreadPriority", "ServiceSpreadingPriority"} <= names
        saa = [custom[n][1] for n in names if custom and n in custom and custom[n][0] == "serviceAntiAffinity"]
        if both and saa and spread:
            raise Unsupported("ServiceSpreadingPriority next to SelectorSpreadPriority and a serviceAntiAffinity "
                              "priority, with spread listers (one auxiliary spreading priority)")
        # a second spreading priority over the services (include/ksim.h ksim_affinity_tables.aux_*)
        aux = ("service_spreading",) if both else (("service_anti_affinity", saa[0]) if len(saa) == 1 else None)
        self.cluster = Cluster.from_objects(nodes, running_pods, self.order, pvs=pvs, pvcs=pvcs,
                                            storage_classes=storage_classes, spread=spread,
                                            spread_services_only="ServiceSpreadingPriority" in names and not both,
                                            aux=aux if spread else None,
                                            service_affinity=svc_aff if "CheckServiceAffinity" in predicates else None)
        self.scheduler = GenericScheduler(self.cluster, predicates, priorities, device=device, mode=mode,
                                          collect_reasons=collect_reasons, label_presence=label_presence,
                                          custom_priorities=custom, service_affinity=svc_aff)

    def run(self) -> Report:
        from .report import ERR_NO_NODES, get_report, simulation_status
        rep = Report()
        names = self.cluster.names
        scal = self.cluster.scalar_names.items
        try:
            nodes, reasons, st = self.scheduler.schedule()
            rep.stats = st
            msgs = [None if w >= 0 else (fit_error_message(len(names), reasons[k], scal) if reasons is not None
                                         else "unschedulable") for k, w in enumerate(nodes)]
        except abi.NoNodesAvailable:
            # ErrNoNodesAvailable (generic_scheduler.go:63-64,124-125) for every pod: nothing is
            # ever bound, so each pod in turn fails the same way and goes through Update
            nodes, msgs = np.full(len(self.order), -1, np.int32), [ERR_NO_NODES] * len(self.order)
        rep.last_node_index = self.scheduler.last_node_index
        outcomes = [(names[w] if w >= 0 else None, m) for w, m in zip(nodes, msgs)]
        for k, (node, msg) in enumerate(outcomes):
            name = self.cluster.pod_names[k]
            if node is not None:
                rep.successful.append((name, node))
            else:
                rep.failed.append((name, msg))
        rep.status = simulation_status(self.order, self.running, outcomes)
        rep.stop_reason = rep.status.stop_reason
        rep.review = get_report(rep.status)
        return rep
