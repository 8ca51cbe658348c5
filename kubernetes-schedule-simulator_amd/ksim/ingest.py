"""Snapshot ingest: Kubernetes-shaped v1.Node / v1.Pod objects → the device layout.

Nodes become a struct-of-arrays table in ascending bytewise name order (so a node index is
its name rank, which is what selectHost's tie order needs).  Strings never reach the
device: label sets, taint sets, scalar resource names, host IPs and protocols are interned
here, and every string comparison the scheduler makes (label selectors, tolerations) is
evaluated once per (pod class, label set / taint set) into bit and byte tables.

Reference semantics implemented here (file:line under vendor/k8s.io/kubernetes/pkg/scheduler/):
- NodeInfo.SetNode (schedulercache/node_info.go:429-448), Resource.Add (:86-109)
- NodeInfo.AddPod for pods already running (node_info.go:318-341, calculateResource :400-412)
- GetResourceRequest (algorithm/predicates/predicates.go:659-697)
- GetNonzeroRequests (algorithm/priorities/util/non_zero.go:38-53)
- isPodBestEffort → GetPodQOS (K/pkg/apis/core/v1/helper/qos/qos.go:39-85)
- GetContainerPorts + HostPortInfo sanitising (util/utils.go:31-155)
- CheckNodeConditionPredicate's condition rules (predicates.go:1534-1568)
- podMatchesNodeLabels (predicates.go:795-838), PodToleratesNodeTaints (:1465-1494),
  ToleratesTaint (vendor/k8s.io/api/core/v1/toleration.go:37-56)
- TaintToleration / NodeAffinity priority map values (priorities/taint_toleration.go:29-73,
  priorities/node_affinity.go:34-75)
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field

import numpy as np

from . import abi, labels, quantity

CPU, MEM, GPU, EPH, PODS = "cpu", "memory", "alpha.kubernetes.io/nvidia-gpu", "ephemeral-storage", "pods"
DEFAULT_MILLI_CPU = 100
DEFAULT_MEMORY = 200 * 1024 * 1024
PREFER_AVOID_ANNOTATION = "scheduler.alpha.kubernetes.io/preferAvoidPods"
# volume sources the volume predicates read (ksim/volumes.py); others never change a verdict
_PREDICATE_VOLUMES = ("gcePersistentDisk", "awsElasticBlockStore", "rbd", "iscsi", "azureDisk",
                      "persistentVolumeClaim")


class Unsupported(abi.KsimUnsupported):
    def __init__(self, msg):
        super().__init__(abi.E_UNSUPPORTED, msg)


def is_scalar_resource(name: str) -> bool:
    """IsScalarResourceName (K/pkg/apis/core/v1/helper/helpers.go:38-96)."""
    if name.startswith("hugepages-"):
        return True
    if "/" not in name or "kubernetes.io/" in name or name.startswith("requests."):
        return False
    return labels.qualified_name("requests." + name)


class ResourceVec:
    """schedulercache.Resource; scalar keeps map *presence* (a zero entry still counts)."""
    __slots__ = ("cpu", "mem", "gpu", "eph", "pods", "scalar")

    def __init__(self):
        self.cpu = self.mem = self.gpu = self.eph = self.pods = 0
        self.scalar = {}

    def add(self, rl):
        for name, q in (rl or {}).items():
            if name == CPU:
                self.cpu += quantity.milli_value(q)
            elif name == MEM:
                self.mem += quantity.value(q)
            elif name == GPU:
                self.gpu += quantity.value(q)
            elif name == PODS:
                self.pods += quantity.value(q)
            elif name == EPH:
                self.eph += quantity.value(q)
            elif is_scalar_resource(name):
                self.scalar[name] = self.scalar.get(name, 0) + quantity.value(q)


def _spec(obj):
    return obj.get("spec") or {}


def _meta(obj):
    return obj.get("metadata") or {}


def _reqs(c):
    return (c.get("resources") or {}).get("requests") or {}


def container_requests(pod):
    """(predicate request, commit delta, nz cpu, nz mem) of a pod."""
    spec = _spec(pod)
    pred, add = ResourceVec(), ResourceVec()
    nzc = nzm = 0
    for c in spec.get("containers") or []:
        r = _reqs(c)
        pred.add(r)
        add.add(r)
        nzc += DEFAULT_MILLI_CPU if CPU not in r else quantity.milli_value(r[CPU])
        nzm += DEFAULT_MEMORY if MEM not in r else quantity.value(r[MEM])
    for c in spec.get("initContainers") or []:
        for name, q in _reqs(c).items():
            if name == MEM:
                pred.mem = max(pred.mem, quantity.value(q))
            elif name == EPH:
                pred.eph = max(pred.eph, quantity.value(q))
            elif name == CPU:
                pred.cpu = max(pred.cpu, quantity.milli_value(q))
            elif name == GPU:
                pred.gpu = max(pred.gpu, quantity.value(q))
            elif is_scalar_resource(name):
                v = quantity.value(q)
                if v > pred.scalar.get(name, 0):
                    pred.scalar[name] = v
    return pred, add, nzc, nzm


def best_effort(pod) -> bool:
    for c in _spec(pod).get("containers") or []:
        res = c.get("resources") or {}
        for rl in (res.get("requests") or {}, res.get("limits") or {}):
            for name, q in rl.items():
                if name in (CPU, MEM) and quantity.positive(q):
                    return False
    return True


def host_ports(pod):
    """[(ip, proto, port)] with HostPortInfo sanitising; port <= 0 never conflicts and is
    never recorded (utils.go:45-48, :101-104), so it is dropped here."""
    out = []
    for c in _spec(pod).get("containers") or []:
        for p in c.get("ports") or []:
            port = int(p.get("hostPort") or 0)
            if port <= 0:
                continue
            out.append((p.get("hostIP") or "0.0.0.0", p.get("protocol") or "TCP", port))
    return out


def tolerates(tol, taint) -> bool:
    eff = tol.get("effect") or ""
    if eff and eff != (taint.get("effect") or ""):
        return False
    key = tol.get("key") or ""
    if key and key != (taint.get("key") or ""):
        return False
    op = tol.get("operator") or ""
    if op in ("", "Equal"):
        return (tol.get("value") or "") == (taint.get("value") or "")
    return op == "Exists"


def has_pod_affinity(pod):
    aff = _spec(pod).get("affinity") or {}
    return aff.get("podAffinity") is not None or aff.get("podAntiAffinity") is not None


def has_predicate_volumes(pod):
    return any(v.get(k) is not None for v in _spec(pod).get("volumes") or [] for k in _PREDICATE_VOLUMES)


def check_pod_supported(pod, where="pod"):
    for v in _spec(pod).get("volumes") or []:
        if sum(v.get(k) is not None for k in _PREDICATE_VOLUMES) > 1:
            raise Unsupported("%s %r: a volume with more than one source" % (where, _meta(pod).get("name")))


@dataclass
class Interner:
    ids: dict = field(default_factory=dict)
    items: list = field(default_factory=list)

    def get(self, key, item=None):
        i = self.ids.get(key)
        if i is None:
            i = len(self.items)
            self.ids[key] = i
            self.items.append(key if item is None else item)
        return i


def _canon(x):
    return json.dumps(x, sort_keys=True, separators=(",", ":"))


class LabelSet(dict):
    """A node label set (a plain dict of labels for every label test) that also carries the
    node's preferAvoidPods controller signatures and — when the cluster interns them
    (Cluster.image_locality) — its image sizes by name: nodes with equal labels but different
    annotations / images are different sets, so NodePreferAvoidPods and ImageLocality are
    functions of (pod class, set)."""

    def __init__(self, labels, avoid=(), images=None):
        super().__init__(labels)
        self.avoid = tuple(avoid)
        self.images = dict(images or {})


def label_set_key(labels, avoid, images=None):
    """Interning key of a label set: the labels' canonical form, plus the avoided controller
    signatures and the image sizes when there are any (so plain sets keep their plain key)."""
    k = _canon(labels)
    if avoid:
        k += "|avoid:" + _canon([list(e) if e is not None else None for e in avoid])
    if images:
        k += "|img:" + _canon(sorted(images.items()))
    return k


MB = 1024 * 1024
MIN_IMG_SIZE, MAX_IMG_SIZE = 23 * MB, 1000 * MB   # image_locality.go:29-33


def node_images(status):
    """totalImageSize's map (image_locality.go:78-84): every name of every listed image → its
    size; a name listed twice keeps the later image's size."""
    out = {}
    for img in (status or {}).get("images") or []:
        for name in img.get("names") or []:
            out[name] = int(img.get("sizeBytes") or 0)
    return out


def image_score(images, node_imgs):
    """ImageLocalityPriorityMap (image_locality.go:39-88): the summed size of the pod's container
    images (spec.containers only) the node lists, bucketed by calculateScoreFromSize."""
    total = sum(node_imgs.get(i, 0) for i in images)
    if total == 0 or total < MIN_IMG_SIZE:
        return 0
    if total >= MAX_IMG_SIZE:
        return 10
    return 10 * (total - MIN_IMG_SIZE) // (MAX_IMG_SIZE - MIN_IMG_SIZE) + 1


def pod_images(spec):
    """The images ImageLocality sums over: spec.containers[*].image, in order (init containers
    are not looked at)."""
    return [c.get("image") or "" for c in spec.get("containers") or []]


def _go_field(obj, name):
    """encoding/json's field lookup: the exact key, else a case-insensitive match; the last
    matching key in document order wins (obj: list of (key, value) pairs)."""
    found, val = False, None
    for k, v in obj:
        if k == name or k.lower() == name.lower():
            found, val = True, v
    return found, val


class _JsonObj(list):
    """A decoded JSON object as its ordered (key, value) pairs."""


def avoid_signatures(annotations):
    """v1helper.GetAvoidPodsFromNodeAnnotations (pkg/apis/core/v1/helper/helpers.go:338-347):
    the preferAvoidPods entries' controller signatures (kind, uid) in order, or None for an entry
    whose podSignature / podController is absent or null.  Any decoding error → no entries (the
    priority then scores the node MaxPriority, node_prefer_avoid_pods.go:53-56); encoding/json
    matches field names exactly or case-insensitively, and a type error anywhere fails the whole
    decode.  evictionTime is only checked to be a string."""
    raw = (annotations or {}).get(PREFER_AVOID_ANNOTATION) or ""
    if not raw:
        return ()
    try:
        doc = json.loads(raw, object_pairs_hook=_JsonObj)
    except ValueError:
        return ()
    if not isinstance(doc, _JsonObj):
        return ()
    ok, lst = _go_field(doc, "preferAvoidPods")
    if not ok or lst is None:
        return ()
    if not isinstance(lst, list) or isinstance(lst, _JsonObj):
        return ()

    def strings_ok(o, names):
        return all((lambda v: v is None or isinstance(v, str))(_go_field(o, n)[1]) for n in names)

    entries, err = [], False
    for e in lst:
        if e is None:
            entries.append(None)
            continue
        if not isinstance(e, _JsonObj) or not strings_ok(e, ("reason", "message", "evictionTime")):
            err = True
            continue
        ok, sig = _go_field(e, "podSignature")
        if not ok or sig is None:
            entries.append(None)
            continue
        if not isinstance(sig, _JsonObj):
            err = True
            continue
        ok, ctl = _go_field(sig, "podController")
        if not ok or ctl is None:
            entries.append(None)
            continue
        if not isinstance(ctl, _JsonObj) or not strings_ok(ctl, ("kind", "uid", "name", "apiVersion")):
            err = True
            continue
        if any(_go_field(ctl, n)[1] is not None and not isinstance(_go_field(ctl, n)[1], bool)
               for n in ("controller", "blockOwnerDeletion")):
            err = True
            continue
        entries.append((_go_field(ctl, "kind")[1] or "", _go_field(ctl, "uid")[1] or ""))
    return () if err else tuple(entries)


def avoid_score(entries, ctrl):
    """CalculateNodePreferAvoidPodsPriorityMap's loop (node_prefer_avoid_pods.go:57-63) for a pod
    whose RC / RS controllerRef is ctrl: 0 at the first entry with the same (kind, uid), else
    MaxPriority.  The reference dereferences a nil podController before reaching later entries:
    Unsupported."""
    for e in entries:
        if e is None:
            raise Unsupported("preferAvoidPods entry without a podController (the reference dereferences nil)")
        if e == tuple(ctrl):
            return 0
    return 10


def avoid_controller(md):
    """The pod's controllerRef as CalculateNodePreferAvoidPodsPriorityMap uses it
    (node_prefer_avoid_pods.go:38-50, priorities/util/util.go:25-36): the first ownerReference with
    controller=true, kept only for ReplicationController / ReplicaSet → (kind, uid), else None."""
    for o in md.get("ownerReferences") or []:
        if o.get("controller") is True:
            if o.get("kind") in ("ReplicationController", "ReplicaSet"):
                return (o.get("kind"), o.get("uid") or "")
            return None
    return None


class Cluster:
    """Node table + pod queue in device layout.  Build with from_objects() or from arrays."""

    def __init__(self):
        self.names = []
        self.index = {}
        self.cols = {}
        self.label_sets = Interner()
        self.taint_sets = Interner()
        self.scalar_names = Interner()
        self.ips = Interner()
        self.protos = Interner()
        self.port_slots = 0
        self.classes = Interner()
        self.class_specs = []
        self.pods = None
        self.pod_ports = np.zeros(0, np.uint64)
        self.pod_scalars = np.zeros(0, abi.SCALAR_DTYPE)
        self.pod_names = []
        self.tables = None
        self.prefer_avoid_nodes = False
        self.node_images = False   # some node lists status.images (ImageLocalityPriority not constant)
        # node images are interned into the label sets and pod images into the classes (what
        # ImageLocalityPriority reads); from_objects turns it on when some node lists images
        self.image_locality = False
        self.bad_affinity_classes = set()   # preferred terms that fail to parse
        self.affinity = None     # inter-pod affinity tables (ksim/affinity.py), None without terms
        self.hard_weight = 10
        self.volume_index = None  # ksim/volumes.py VolumeIndex when a pod has predicate volumes
        self.volumes = None       # its device tables (volumes.build_tables)
        self.spread_active = False
        self.aux = None           # the auxiliary spreading priority (from_objects(aux=...))
        self.aux_sels = []
        self.aux_active = False   # some queued pod has a counted auxiliary pair
        self.svc_labels = None    # CheckServiceAffinity's labels the cluster was built for
        self.svc_any = False      # a service selects some queued pod
        self.svc_miss = []
        self.svc_active = False   # some queued pod needs the lender check

    # ------------------------------------------------------------------ nodes
    @classmethod
    def from_objects(cls, nodes, running_pods=(), pods=(), port_slots=None, hard_weight=10, pvs=(), pvcs=(),
                     storage_classes=(), max_vols=None, vol_slots=None, spread=None, spread_services_only=False,
                     image_locality=None, aux=None, service_affinity=None):
        """nodes / running_pods / pods: Kubernetes-shaped dicts; pods are in SCHEDULING
        order (the caller resolves the simulator's LIFO queue).  hard_weight:
        hardPodAffinitySymmetricWeight (the simulator's 10, or a Policy's).  pvs / pvcs /
        storage_classes: what the PV / PVC / StorageClass listers hold (the simulator's are empty);
        max_vols: the MaxPD limits (EBS, GCE PD, Azure Disk), default KUBE_MAX_PD_VOLS / getMaxVols.
        spread: ksim.spread.SpreadListers (services / RCs / RSs / StatefulSets) for SelectorSpread
        (spread_services_only: ServiceSpreadingPriority's services-only form); None: the simulator's
        empty listers.  image_locality: intern node / pod images (what ImageLocalityPriority reads;
        default: when some node lists status.images).  aux: a second counted spreading priority over
        `spread`'s services (include/ksim.h ksim_affinity_tables.aux_*): ("service_spreading",) —
        ServiceSpreadingPriority next to SelectorSpreadPriority — or ("service_anti_affinity", label),
        a Policy's serviceAntiAffinity priority; None: neither.  service_affinity: CheckServiceAffinity's
        labels (a Policy's serviceAffinity argument) — with `spread`'s services, pods a service selects
        whose nodeSelector lacks some of them get the lender check (include/ksim.h
        ksim_affinity_tables.svc_*)."""
        self = cls()
        self.hard_weight = int(hard_weight)
        self.image_locality = (any((x.get("status") or {}).get("images") for x in nodes) if image_locality is None
                               else bool(image_locality))
        self.ips.get("0.0.0.0")     # id 0 = wildcard
        self.protos.get("TCP")      # id 0 = default protocol
        nodes = sorted(nodes, key=lambda n: _meta(n).get("name", "").encode())
        n = len(nodes)
        self.names = [_meta(x).get("name", "") for x in nodes]
        if len(set(self.names)) != n:
            raise abi.KsimError(abi.E_INVAL, "duplicate node names")
        self.index = {nm: i for i, nm in enumerate(self.names)}
        running = [p for p in running_pods if _spec(p).get("nodeName") in self.index]
        for p in running:
            check_pod_supported(p, "running pod")
        with_pod_affinity = any(has_pod_affinity(p) for p in list(running_pods) + list(pods))
        self.spread_sels = [spread.selectors(p, spread_services_only) if spread else [] for p in pods]
        self.spread_active = any(self.spread_sels)
        self.aux = aux
        self.aux_sels = [spread.selectors(p, True) if (spread and aux) else [] for p in pods]
        if aux and aux[0] == "service_anti_affinity":
            for p, s in zip(pods, self.aux_sels):
                if len(s) > 1:
                    # getFirstServiceSelector takes the ServiceLister's first (selector_spreading.go:
                    # 232-245), an informer-cache order: ambiguous unless one service selects the pod
                    raise Unsupported("ServiceAntiAffinity: %d services select pod %r (the service lister's order "
                                      "decides)" % (len(s), _meta(p).get("name")))
        self.aux_active = any(self.aux_sels)
        # CheckServiceAffinity with services (predicates.go:980-1011): per queued pod the missing
        # labels when a service selects it, else 0
        self.svc_labels = list(service_affinity) if service_affinity is not None else None
        self.svc_any = bool(spread) and any(spread.selectors(p, True) for p in pods)
        self.svc_miss = [0] * len(pods)
        if self.svc_labels is not None and spread:
            if len(self.svc_labels) > abi.SVC_LABELS:
                raise Unsupported("CheckServiceAffinity with more than %d labels and services" % abi.SVC_LABELS)
            for k, p in enumerate(pods):
                sel = _spec(p).get("nodeSelector") or {}
                miss = sum(1 << l for l, name in enumerate(self.svc_labels) if name not in sel)
                if miss and spread.selectors(p, True):
                    self.svc_miss[k] = miss
            need = {(_meta(p).get("namespace", ""), _canon(_meta(p).get("labels") or {})): p
                    for p, m in zip(pods, self.svc_miss) if m}
            for q in running_pods:
                if not _spec(q).get("nodeName") or _spec(q).get("nodeName") in self.index:
                    continue
                qm = _meta(q)
                for (ns, _), p in need.items():
                    lab = _meta(p).get("labels") or {}
                    if qm.get("namespace", "") == ns and all((qm.get("labels") or {}).get(k) == v for k, v in lab.items()):
                        # GetNodeInfo errs for a lender outside the node lister (predicates.go:1003-1006)
                        raise Unsupported("CheckServiceAffinity: a cached pod with pod %r's labels is bound to a node "
                                          "outside the snapshot" % _meta(p).get("name"))
        self.svc_active = any(self.svc_miss)
        with_affinity = with_pod_affinity or self.spread_active or self.aux_active or self.svc_active
        if with_pod_affinity and len(running) != len([p for p in running_pods if _spec(p).get("nodeName")]):
            # the reference caches them under a node-less NodeInfo: its affinity metadata then
            # errors and the predicate takes another path (metadata.go:106-109)
            raise Unsupported("running pods bound to nodes outside the snapshot, with inter-pod affinity terms")
        # scalar columns: every scalar name any node or pod mentions
        for x in nodes:
            for name in ((x.get("status") or {}).get("allocatable") or {}):
                if is_scalar_resource(name):
                    self.scalar_names.get(name)
        compiled = []
        for p in list(running) + list(pods):
            pred, add, nzc, nzm = container_requests(p)
            for name in list(pred.scalar) + list(add.scalar):
                self.scalar_names.get(name)
            compiled.append((pred, add, nzc, nzm))
        if len(self.scalar_names.items) > abi.MAX_SCALAR:
            raise Unsupported("more than %d scalar resources" % abi.MAX_SCALAR)
        S = len(self.scalar_names.items)
        z64 = lambda: np.zeros(n, np.int64)
        c = dict(alloc_cpu=z64(), alloc_mem=z64(), alloc_gpu=z64(), alloc_eph=z64(),
                 allowed_pods=np.zeros(n, np.int32), flags=np.zeros(n, np.uint32),
                 label_set=np.zeros(n, np.int32), taint_set=np.zeros(n, np.int32),
                 alloc_scalar=np.zeros((S, n), np.int64), req_cpu=z64(), req_mem=z64(), req_gpu=z64(),
                 req_eph=z64(), nz_cpu=z64(), nz_mem=z64(), pod_count=np.zeros(n, np.int32),
                 req_scalar=np.zeros((S, n), np.int64))
        node_taints = []
        for i, x in enumerate(nodes):
            ns = node_static(x)
            c["alloc_cpu"][i], c["alloc_mem"][i], c["alloc_gpu"][i], c["alloc_eph"][i] = ns.alloc
            c["allowed_pods"][i] = ns.allowed
            for name, v in ns.scalar.items():
                c["alloc_scalar"][self.scalar_names.ids[name], i] = v
            c["flags"][i] = ns.flags
            imgs = ns.images if self.image_locality else None
            c["label_set"][i] = self.label_sets.get(label_set_key(ns.labels, ns.prefer_avoid, imgs),
                                                    LabelSet(ns.labels, ns.prefer_avoid, imgs))
            c["taint_set"][i] = self.taint_sets.get(_canon(ns.taints), ns.taints)
            self.prefer_avoid_nodes |= bool(ns.prefer_avoid)
            self.node_images |= bool((x.get("status") or {}).get("images"))
            node_taints.append(ns.taints)
        # running pods: NodeInfo.AddPod
        used_ports = [dict() for _ in range(n)]
        for p, (pred, add, nzc, nzm) in zip(running, compiled[:len(running)]):
            i = self.index[_spec(p)["nodeName"]]
            c["req_cpu"][i] += add.cpu
            c["req_mem"][i] += add.mem
            c["req_gpu"][i] += add.gpu
            c["req_eph"][i] += add.eph
            for name, v in add.scalar.items():
                c["req_scalar"][self.scalar_names.ids[name], i] += v
            c["nz_cpu"][i] += nzc
            c["nz_mem"][i] += nzm
            c["pod_count"][i] += 1
            for ip, proto, port in host_ports(p):
                used_ports[i][abi_port_key(self.ips.get(ip), self.protos.get(proto), port)] = True
        self.cols = c
        # pod queue
        self._affinity_ok = with_affinity
        if any(has_predicate_volumes(p) for p in list(running) + list(pods)):
            from .volumes import VolumeIndex
            self.volume_index = VolumeIndex(pvs, pvcs, storage_classes)
        self._compile_pods(list(pods), compiled[len(running):])
        if with_affinity:
            self._build_affinity(nodes, running, list(pods))
        # port slots: enough for everything that could land on one node
        need = max([len(u) for u in used_ports] + [0])
        if self.pods is not None and len(self.pods):
            per_pod = int(self.pods["port_cnt"].max()) if len(self.pods) else 0
            if per_pod:
                distinct = len(set(int(k) for k in self.pod_ports))
                need += distinct
        self.port_slots = int(port_slots if port_slots is not None else max(need, 0))
        P = self.port_slots
        ports = np.zeros((P, n), np.uint64)
        pc = np.zeros(n, np.int32)
        for i, u in enumerate(used_ports):
            if len(u) > P:
                raise abi.KsimError(abi.E_INVAL, "port_slots too small for running pods")
            for s, k in enumerate(u):
                ports[s, i] = k
            pc[i] = len(u)
        c["ports"], c["port_count"] = ports, pc
        self._build_tables()
        if self.volume_index is not None:
            from .volumes import build_tables
            mounts = self.volume_index.node_slots(n, [(self.index[_spec(p)["nodeName"]], p) for p in running])
            self.volumes = build_tables(self.volume_index, n, mounts, self.pods["vol_class"] if self.pods is not None else (),
                                        self.label_sets.items, max_vols, vol_slots)
        return self

    # ------------------------------------------------------------------- pods
    def _compile_pods(self, pods, compiled):
        m = len(pods)
        arr = np.zeros(m, abi.POD_DTYPE)
        ports, scalars = [], []
        self.pod_names = []
        for k, (p, cr) in enumerate(zip(pods, compiled)):
            self.pod_names.append(_meta(p).get("name", ""))
            self.encode_pod(p, cr, arr[k], ports, scalars)
        self.pods = arr
        self.pod_ports = np.array(ports, np.uint64)
        self.pod_scalars = np.array(scalars, abi.SCALAR_DTYPE) if scalars else np.zeros(0, abi.SCALAR_DTYPE)

    def encode_pod(self, p, compiled, row, ports, scalars, index=None):
        """One pod → a ksim_pod record `row` (a POD_DTYPE element); its host-port keys and scalar
        requests are appended to `ports` / `scalars` (offsets into those lists).  Interns the
        pod's class (nodeSelector, node affinity, tolerations) and any new IP / protocol.
        `index` maps spec.nodeName to a name rank (default: the cluster's own index)."""
        pred, add, nzc, nzm = compiled
        check_pod_supported(p)
        if has_pod_affinity(p) and not getattr(self, "_affinity_ok", False):
            raise Unsupported("pod %r: inter-pod affinity needs the cluster's affinity tables (ClusterCapacity / "
                              "GenericScheduler)" % _meta(p).get("name"))
        spec, md = _spec(p), _meta(p)
        row["req_cpu"], row["req_mem"], row["req_gpu"], row["req_eph"] = pred.cpu, pred.mem, pred.gpu, pred.eph
        row["add_cpu"], row["add_mem"], row["add_gpu"], row["add_eph"] = add.cpu, add.mem, add.gpu, add.eph
        row["nz_cpu"], row["nz_mem"] = nzc, nzm
        flags = 0
        if pred.cpu or pred.mem or pred.gpu or pred.eph or pred.scalar:
            flags |= abi.POD_ANY_REQUEST
        if best_effort(p):
            flags |= abi.POD_BEST_EFFORT
        nn = spec.get("nodeName") or ""
        idx = self.index if index is None else index
        row["host"] = -1 if not nn else idx.get(nn, -2)
        ctrl = avoid_controller(md)
        imgs = pod_images(spec) if self.image_locality else None
        cspec = spec if ctrl is None else dict(spec, __ctrl=ctrl)
        if imgs and any(imgs):
            cspec = dict(cspec, __img=imgs)
        row["cls"] = self.classes.get(pod_class_key(spec, ctrl, imgs), cspec)
        row["flags"] = flags
        hp = host_ports(p)
        row["port_off"], row["port_cnt"] = len(ports), len(hp)
        for ip, proto, port in hp:
            ports.append(abi_port_key(self.ips.get(ip), self.protos.get(proto), port))
        row["scalar_off"], row["scalar_cnt"] = len(scalars), len(pred.scalar)
        for name, v in pred.scalar.items():
            scalars.append((self.scalar_names.ids[name], 0, v, add.scalar.get(name, 0)))
        if has_predicate_volumes(p):
            if self.volume_index is None:
                raise Unsupported("pod %r: volumes need the cluster's volume tables (ClusterCapacity / "
                                  "GenericScheduler)" % md.get("name"))
            row["vol_class"] = self.volume_index.vclass(p)

    def _build_affinity(self, nodes, running, pods):
        """Inter-pod affinity tables over every pod's identity and terms (ksim/affinity.py); the
        queued descriptors get their aff_ident / aff_class."""
        from .affinity import ZONE_KEY, AffinityIndex
        idx = AffinityIndex([_meta(x).get("labels") for x in nodes], self.hard_weight)
        allp = list(running) + list(pods)
        idents = [idx.ident(p) for p in allp]
        sels = [()] * len(running) + list(self.spread_sels)
        asels = [()] * len(running) + list(self.aux_sels)
        if self.aux_active:
            idx.set_aux(abi.AUX_SPREAD, ZONE_KEY) if self.aux[0] == "service_spreading" else \
                idx.set_aux(abi.AUX_SERVICE_ANTI, self.aux[1])
        svcs = [None] * len(allp)
        if self.svc_active:
            idx.set_svc(self.svc_labels)
            k0 = len(running)
            for k, m in enumerate(self.svc_miss):
                if m:
                    svcs[k0 + k] = idx.svc_class(allp[k0 + k], m)
        aclasses = [idx.aclass(p, s, a, v) for p, s, a, v in zip(allp, sels, asels, svcs)]
        run_nodes = [self.index[_spec(p)["nodeName"]] for p in running]
        self.affinity, remap = idx.build(run_nodes, idents, aclasses)
        k = len(running)
        if len(pods):
            self.pods["aff_ident"] = remap[np.asarray(idents[k:], np.int64)]
            self.pods["aff_class"] = np.asarray(aclasses[k:], np.int32) + 1

    # ----------------------------------------------------------------- tables
    def _build_tables(self):
        if not self.label_sets.items:   # an empty cluster still has well-formed tables
            self.label_sets.get(_canon({}), {})
        if not self.taint_sets.items:
            self.taint_sets.get(_canon([]), [])
        self.tables, need, bad = build_class_tables(self.label_sets.items, self.taint_sets.items,
                                                    self.classes.items or [{}])
        self.bad_affinity_classes |= bad
        if self.pods is not None and len(self.pods):
            self.pods["flags"] |= need[self.pods["cls"]]

    # ------------------------------------------------------------ ABI structs
    def node_table(self):
        c = self.cols
        t = abi.NodeTable()
        t.n_nodes = len(self.names) if self.names else len(c["alloc_cpu"])
        t.n_scalar = c["alloc_scalar"].shape[0]
        t.port_slots = self.port_slots
        for name, ct in (("alloc_cpu", abi.C.c_int64), ("alloc_mem", abi.C.c_int64), ("alloc_gpu", abi.C.c_int64),
                         ("alloc_eph", abi.C.c_int64), ("allowed_pods", abi.C.c_int32), ("flags", abi.C.c_uint32),
                         ("label_set", abi.C.c_int32), ("taint_set", abi.C.c_int32), ("alloc_scalar", abi.C.c_int64),
                         ("req_cpu", abi.C.c_int64), ("req_mem", abi.C.c_int64), ("req_gpu", abi.C.c_int64),
                         ("req_eph", abi.C.c_int64), ("nz_cpu", abi.C.c_int64), ("nz_mem", abi.C.c_int64),
                         ("pod_count", abi.C.c_int32), ("req_scalar", abi.C.c_int64), ("ports", abi.C.c_uint64),
                         ("port_count", abi.C.c_int32)):
            a = c.get(name)
            if a is not None:
                a = np.ascontiguousarray(a)
                c[name] = a
                setattr(t, name, abi.ptr(a, ct))
        return t

    def class_tables(self, na_add=None):
        return class_tables_struct(self.tables, na_add)

    @property
    def n_nodes(self):
        return len(self.cols["alloc_cpu"])

    def shard(self, lo, hi):
        """The name-rank range [lo, hi) of the node table with the same pods and interned
        tables (node-sharded mode: rank r loads its contiguous shard, ksim_shard_setup)."""
        import copy
        sub = copy.copy(self)
        if self.affinity is not None:
            sub.affinity = _shard_affinity(self.affinity, lo, hi)
        if self.volumes is not None:
            v = dict(self.volumes)
            if v.get("slots") is not None:
                v["slots"] = np.ascontiguousarray(v["slots"][:, lo:hi])
                v["slot_count"] = np.ascontiguousarray(v["slot_count"][lo:hi])
            v["n_nodes"] = hi - lo
            sub.volumes = v
        sub.cols = {k: (np.ascontiguousarray(v[..., lo:hi]) if isinstance(v, np.ndarray) else v)
                    for k, v in self.cols.items()}
        sub.names = list(self.names[lo:hi]) if self.names else self.names
        sub.index = {}
        return sub


def _shard_affinity(d, lo, hi):
    """The affinity tables of node-sharded rank [lo, hi) (SURVEY.md §8e Phase A): every counted pair,
    carried term and term key must be node-like (each domain holds at most one node: the node
    pseudo key, a unique hostname label), so a commit changes counts on its own rank only: the
    node pseudo key's domains become the shard's node indices (its count segments sliced), other
    node-like keys keep their global domain ids and count arrays; the domain columns are sliced.  The zone key
    only groups the spread reduce's counts (exchanged across ranks in pass A).  Other keys — a
    domain several ranks share — are refused."""
    dom = np.asarray(d["dom"])
    K = dom.shape[0]
    nodelike = np.zeros(K, bool)
    for k in range(K):
        row = dom[k][dom[k] >= 0]
        nodelike[k] = len(np.unique(row)) == len(row)
    used = set(int(x) for x in np.asarray(d["pair_key"])[:int(d["n_pair"])]) | \
        set(int(x) for x in np.asarray(d["carry_key"])[:int(d["n_carry"])])
    terms = np.asarray(d["terms"])[:int(d.get("n_terms", len(d["terms"])))]
    for t in terms:
        if int(t["kind"]) != abi.AFF_PREFERRED:
            used.add(int(t["gate_key"]))
    bad = sorted(k for k in used if not nodelike[k])
    if bad:
        raise Unsupported("node-sharded scheduling of inter-pod affinity / spread terms over topology domains several "
                          "nodes share (keys %s)" % bad)
    if d.get("svc_on"):
        raise Unsupported("node-sharded scheduling with CheckServiceAffinity lenders")
    # the auxiliary priority: its pair is node-keyed (a rank's own counts), its key only groups the
    # fit nodes' counts — domain sums exchanged across ranks in pass A, like the spread zones
    if d.get("aux_pair") is not None and int(np.asarray(d["n_dom"])[int(d["aux_key"])]) > abi.SHARD_MAX_AUX_DOMAINS:
        raise Unsupported("node-sharded scheduling of the auxiliary priority over more than %d domains"
                          % abi.SHARD_MAX_AUX_DOMAINS)
    if int(d["zone_key"]) >= 0 and int(np.asarray(d["n_dom"])[int(d["zone_key"])]) > abi.SHARD_MAX_ZONES:
        raise Unsupported("node-sharded scheduling of spread pods over more than %d zones" % abi.SHARD_MAX_ZONES)
    out = dict(d)
    n = hi - lo
    sdom = np.ascontiguousarray(dom[:, lo:hi])
    # the node pseudo key (1) becomes the shard's own: node i's domain is i (the kernels read a
    # node-key pair's count at the node's index), its pairs' / carried terms' segments sliced to
    # [lo, hi); every other key keeps its global domain ids
    sdom[1] = np.arange(n, dtype=sdom.dtype)
    n_dom = np.asarray(d["n_dom"]).copy()
    n_dom[1] = n

    def reslice(keys, offs, arr, m):
        new_off = np.zeros(m, np.int64)
        parts, o = [], 0
        for c in range(m):
            k, a = int(keys[c]), int(offs[c])
            seg = arr[a + lo:a + hi] if k == 1 else arr[a:a + int(np.asarray(d["n_dom"])[k])]
            new_off[c] = o
            parts.append(seg)
            o += len(seg)
        flat = np.concatenate(parts) if parts else arr[:0]
        return new_off, np.ascontiguousarray(flat if len(flat) else np.zeros(1, arr.dtype))

    P, E = int(d["n_pair"]), int(d["n_carry"])
    out["pair_off"], out["cnt"] = reslice(np.asarray(d["pair_key"]), np.asarray(d["pair_off"]), np.asarray(d["cnt"]), P)
    out["carry_off"], out["carried"] = reslice(np.asarray(d["carry_key"]), np.asarray(d["carry_off"]),
                                               np.asarray(d["carried"]), E)
    out["dom"], out["n_dom"], out["n_nodes"] = sdom, n_dom.astype(np.int32), n
    return out


@dataclass
class NodeStatic:
    alloc: tuple          # allocatable cpu (milli), memory, gpu, ephemeral
    allowed: int          # allocatable pods
    scalar: dict          # allocatable scalar resources
    flags: int            # KSIM_N_* condition bits
    labels: dict
    taints: list
    prefer_avoid: tuple  # preferAvoidPods controller signatures (avoid_signatures)
    mem_pressure: object  # status of the last MemoryPressure condition (None: absent)
    disk_pressure: object
    images: dict = None   # status.images sizes by name (node_images)


def node_static(x, prev_mem=None, prev_disk=None):
    """NodeInfo.SetNode (node_info.go:429-448) + the conditions CheckNodeConditionPredicate reads
    (predicates.go:1534-1568).  SetNode overwrites the pressure status only when the node carries
    that condition, so an update keeps the previous one otherwise (prev_mem / prev_disk)."""
    st, sp, md = x.get("status") or {}, _spec(x), _meta(x)
    r = ResourceVec()
    r.add(st.get("allocatable") or {})
    f = 0
    mem, disk = prev_mem, prev_disk
    seen = {}
    for cond in st.get("conditions") or []:
        t, s = cond.get("type"), cond.get("status")
        bit = 0
        if t == "Ready" and s != "True":
            bit = abi.N_NOT_READY
        elif t == "OutOfDisk" and s != "False":
            bit = abi.N_OUT_OF_DISK
        elif t == "NetworkUnavailable" and s != "False":
            bit = abi.N_NET_UNAVAIL
        if bit:
            # CheckNodeConditionPredicate appends one reason per failing entry and FitError counts
            # each: a repeated failing condition would count twice, which one bit cannot say
            if seen.get(bit):
                raise Unsupported("node %r: repeated failing %s condition" % (md.get("name"), t))
            seen[bit] = True
            f |= bit
        if t == "MemoryPressure":    # SetNode keeps the last such condition
            mem = s
        elif t == "DiskPressure":
            disk = s
    if mem == "True":
        f |= abi.N_MEM_PRESSURE
    if disk == "True":
        f |= abi.N_DISK_PRESSURE
    if sp.get("unschedulable"):
        f |= abi.N_UNSCHEDULABLE
    taints = [{"key": t.get("key") or "", "value": t.get("value") or "", "effect": t.get("effect") or ""}
              for t in (sp.get("taints") or [])]
    return NodeStatic((r.cpu, r.mem, r.gpu, r.eph), r.pods, dict(r.scalar), f, dict(md.get("labels") or {}), taints,
                      avoid_signatures(md.get("annotations")), mem, disk, node_images(st))


def pod_class_key(spec, ctrl=None, images=None):
    """Pods whose nodeSelector, node affinity and tolerations are equal share a class; an RC / RS
    controllerRef (NodePreferAvoidPods' input) and the container images (ImageLocality's, when
    the cluster interns them) are part of the class when present."""
    k = {"ns": spec.get("nodeSelector") or {}, "na": (spec.get("affinity") or {}).get("nodeAffinity"),
         "tol": spec.get("tolerations") or []}
    if ctrl is not None:
        k["ctrl"] = list(ctrl)
    if images and any(images):
        k["img"] = list(images)
    return _canon(k)


def build_class_tables(label_items, taint_items, specs):
    """Per pod class × label set / taint set: podMatchesNodeLabels (predicates.go:795-838),
    PodToleratesNodeTaints (:1465-1494, NoSchedule + NoExecute; NoExecute only), the
    TaintToleration map value (intolerable PreferNoSchedule taints, taint_toleration.go:29-73)
    and the NodeAffinity map value (preferred terms' weight, node_affinity.go:34-75) grouped
    into reduce classes.  Returns (tables, POD_NEED_* flags per class, classes whose preferred
    terms fail to parse)."""
    L, T = len(label_items), len(taint_items)
    Cn = len(specs)
    lw, tw = (L + 31) // 32, (T + 31) // 32
    sel = np.zeros((Cn, lw), np.uint32)
    tok = np.zeros((Cn, tw), np.uint32)
    nok = np.zeros((Cn, tw), np.uint32)
    ttc = np.zeros((Cn, T), np.uint8)
    nac = np.zeros((Cn, L), np.uint8)
    ntt = np.ones(Cn, np.int32)
    nna = np.ones(Cn, np.int32)
    tvs, avs = [], []  # per class: its distinct TaintToleration / NodeAffinity values
    na_w = np.zeros((Cn, L), np.int64)   # preferred node-affinity weight per (class, label set)
    na_p = np.full((Cn, L), 10, np.int64)  # NodePreferAvoidPods map score per (class, label set)
    im_s = np.zeros((Cn, L), np.int64)     # ImageLocality map score per (class, label set)
    need = np.zeros(Cn, np.uint32)
    pa_split = False
    bad = set()
    for k, spec in enumerate(specs):
        tols = spec.get("tolerations") or []
        prefer_tols = [t for t in tols if (t.get("effect") or "") in ("", "PreferNoSchedule")]
        all_sel = all_taint = True
        weights = []
        ctrl = spec.get("__ctrl")
        imgs = spec.get("__img")
        pas = []
        for li, lab in enumerate(label_items):
            # CalculateNodePreferAvoidPodsPriorityMap (node_prefer_avoid_pods.go:32-68)
            pas.append(10 if ctrl is None else avoid_score(getattr(lab, "avoid", ()), ctrl))
            if imgs:
                im_s[k, li] = image_score(imgs, getattr(lab, "images", None) or {})
            ok = labels.pod_matches_node_labels(spec, lab)
            if ok:
                sel[k, li >> 5] |= np.uint32(1 << (li & 31))
            all_sel &= ok
            try:
                weights.append(labels.preferred_weight(spec, lab))
            except labels.SelectorError:
                # CalculateNodeAffinityPriorityMap returns an error: only fatal when
                # NodeAffinityPriority is configured (checked by the scheduler layer)
                bad.add(k)
                weights.append(0)
        counts = []
        for ti, taints in enumerate(taint_items):
            ok = all(any(tolerates(t, x) for t in tols) for x in taints
                     if x["effect"] in ("NoSchedule", "NoExecute"))
            ok2 = all(any(tolerates(t, x) for t in tols) for x in taints if x["effect"] == "NoExecute")
            if ok:
                tok[k, ti >> 5] |= np.uint32(1 << (ti & 31))
            if ok2:
                nok[k, ti >> 5] |= np.uint32(1 << (ti & 31))
            all_taint &= ok and ok2
            counts.append(sum(1 for x in taints if x["effect"] == "PreferNoSchedule"
                              and not any(tolerates(t, x) for t in prefer_tols)))
        tv = sorted(set(counts))
        av = sorted(set(weights))
        if len(tv) * len(av) > abi.MAX_WIDE:
            # NormalizeReduce takes any number of values (reduce.go:29-64); one pod's reduce classes are
            # bounded by the launch form's wide decision (a product above 16 decides there)
            raise Unsupported("pod class needs %d x %d reduce classes (> %d)" % (len(tv), len(av), abi.MAX_WIDE))
        ntt[k], nna[k] = len(tv), len(av)
        tvs.append(tv)
        avs.append(av)
        ttc[k, :] = [tv.index(x) for x in counts]
        nac[k, :] = [av.index(x) for x in weights]
        # raw per-label-set inputs of the NodeAffinity class dimension, for a scheduler whose
        # policy also weighs NodePreferAvoidPods (scheduler.class_tables_for re-keys the classes)
        na_w[k, :] = weights
        na_p[k, :] = pas
        pa_split |= len(set(pas)) > 1
        f = 0
        if not all_sel:
            f |= abi.POD_NEED_SELECTOR
        if not all_taint:
            f |= abi.POD_NEED_TAINTS
        need[k] = f
    # the value rows: 16 wide, or as wide as the widest class's larger dimension
    W = max([abi.MAX_RCLASS] + [max(len(a), len(b)) for a, b in zip(tvs, avs)])
    ttv = np.zeros((Cn, W), np.int64)
    nav = np.zeros((Cn, W), np.int64)
    for k, (tv, av) in enumerate(zip(tvs, avs)):
        ttv[k, :len(tv)] = tv
        nav[k, :len(av)] = av
    tables = dict(n_classes=Cn, n_label_sets=L, n_taint_sets=T, sel_ok=sel, taint_ok=tok, noexec_ok=nok,
                  tt_class=ttc, na_class=nac, n_tt=ntt, n_na=nna, tt_val=ttv, na_val=nav, na_w=na_w, na_p=na_p,
                  pa_split=pa_split, im_s=im_s)
    return tables, need, bad


def class_tables_struct(d, na_add=None):
    """ksim_class_tables over the arrays of a tables dict (kept alive by the dict); na_add: the
    weighted NodePreferAvoidPods addends per NodeAffinity class (scheduler.prefer_avoid_add)."""
    t = abi.ClassTables()
    t.n_classes, t.n_label_sets, t.n_taint_sets = d["n_classes"], d["n_label_sets"], d["n_taint_sets"]
    for name, ct in (("sel_ok", abi.C.c_uint32), ("taint_ok", abi.C.c_uint32), ("noexec_ok", abi.C.c_uint32),
                     ("tt_class", abi.C.c_uint8), ("na_class", abi.C.c_uint8), ("n_tt", abi.C.c_int32),
                     ("n_na", abi.C.c_int32), ("tt_val", abi.C.c_int64), ("na_val", abi.C.c_int64)):
        d[name] = np.ascontiguousarray(d[name])
        setattr(t, name, abi.ptr(d[name], ct))
    if na_add is not None:
        d["na_add"] = np.ascontiguousarray(na_add, np.int64)
        t.na_add = abi.ptr(d["na_add"], abi.C.c_int64)
    if d.get("svc_ok") is not None:
        d["svc_ok"] = np.ascontiguousarray(d["svc_ok"], np.uint32)
        t.svc_ok = abi.ptr(d["svc_ok"], abi.C.c_uint32)
    W = d["tt_val"].shape[1]  # one row width for every value array (ABI 7)
    assert d["na_val"].shape[1] == W and (na_add is None or np.asarray(na_add).shape[1] == W)
    t.val_width = W if W != abi.MAX_RCLASS else 0
    return t


def abi_port_key(ip_id, proto_id, port):
    return (int(ip_id) << 40) | (int(proto_id) << 32) | (int(port) & 0xFFFFFFFF)
