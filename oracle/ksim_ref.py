"""ORACLE — test infrastructure only.  Never imported by the product path.

Object-level, pure-Python restatement of the vendored kube-scheduler v1.10 per-pod
scheduling cycle that xiaoxubeii/kubernetes-schedule-simulator drives, written for
small cases (a few hundred nodes / pods).  It works on Kubernetes-shaped dicts
(``v1.Node`` / ``v1.Pod`` JSON), independent of the product's interning/SoA
ingest, so that parity tests exercise the whole product path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker.

Citation aliases (paths relative to the reference tree):
  S/  = vendor/k8s.io/kubernetes/pkg/scheduler/
  K/  = vendor/k8s.io/kubernetes/
  AM/ = vendor/k8s.io/apimachinery/

Parity pinning: each function below is checked against the golden vectors
transcribed from the reference's own Go tests (tests/golden/, see
tests/golden/make_golden.py).  The Go toolchain is absent from this image, so the
reference itself cannot be run.
"""
from __future__ import annotations

import math
import functools
import re
import os
from fractions import Fraction

# --------------------------------------------------------------------------
# Quantity  (AM/pkg/api/resource/quantity.go:157-400 parse, :695-713 Value)
# --------------------------------------------------------------------------
_BIN = {"Ki": 10, "Mi": 20, "Gi": 30, "Ti": 40, "Pi": 50, "Ei": 60}
_DEC = {"n": -9, "u": -6, "m": -3, "": 0, "k": 3, "M": 6, "G": 9, "T": 12, "P": 15, "E": 18}
_QRE = re.compile(r"^([+-]?)([0-9]*)(?:\.([0-9]*))?(.*)$")


def parse_quantity(s) -> Fraction:
    """Exact value of a Quantity string, rounded up to 1e-9 (quantity.go:365-380).  A pure
    function of its argument, memoised (the large parity tests re-parse the same strings for
    every node evaluation)."""
    if isinstance(s, (int,)):
        return Fraction(s)
    return _parse_quantity_str(str(s))


@functools.lru_cache(maxsize=65536)
def _parse_quantity_str(s) -> Fraction:
    if s == "":
        raise ValueError("quantity: empty")
    m = _QRE.match(s)
    if not m:
        raise ValueError("quantity: bad format %r" % s)
    sign, num, den, suf = m.group(1), m.group(2), m.group(3) or "", m.group(4)
    if num == "" and den == "":
        raise ValueError("quantity: no digits %r" % s)
    mant = Fraction(int(num or "0")) + (Fraction(int(den), 10 ** len(den)) if den else 0)
    if suf in _BIN:
        v = mant * (2 ** _BIN[suf])
    elif suf in _DEC:
        v = mant * Fraction(10) ** _DEC[suf]
    elif suf[:1] in ("e", "E") and re.fullmatch(r"[eE][+-]?[0-9]+", suf):
        v = mant * Fraction(10) ** int(suf[1:])
    else:
        raise ValueError("quantity: bad suffix %r" % s)
    # round non-zero values up to the nano scale (quantity.go:365-372)
    nano = v * 10 ** 9
    if nano.denominator != 1:
        v = Fraction(math.ceil(nano), 10 ** 9)
    return -v if sign == "-" else v


@functools.lru_cache(maxsize=65536)
def q_value(s) -> int:
    """Quantity.Value(): ceil(q) (quantity.go:695-713, ScaledValue rounds up)."""
    return math.ceil(parse_quantity(s))


@functools.lru_cache(maxsize=65536)
def q_milli(s) -> int:
    """Quantity.MilliValue(): ceil(q*1000)."""
    return math.ceil(parse_quantity(s) * 1000)


# --------------------------------------------------------------------------
# Resource (S/schedulercache/node_info.go:66-109)
# --------------------------------------------------------------------------
CPU, MEM, GPU, EPH, PODS = "cpu", "memory", "alpha.kubernetes.io/nvidia-gpu", "ephemeral-storage", "pods"


def is_scalar_resource_name(name: str) -> bool:
    """IsScalarResourceName (K/pkg/apis/core/v1/helper/helpers.go:38-96):
    extended (has '/', not in *kubernetes.io/, not requests.*, and
    'requests.'+name is a qualified name) or hugepages-*."""
    if name.startswith("hugepages-"):
        return True
    if "/" not in name or "kubernetes.io/" in name or name.startswith("requests."):
        return False
    return valid_label_key("requests." + name)


class Resource:
    __slots__ = ("cpu", "mem", "gpu", "eph", "pods", "scalar")

    def __init__(self):
        self.cpu = self.mem = self.gpu = self.eph = self.pods = 0
        self.scalar = {}

    def add(self, rl: dict):
        """Resource.Add (node_info.go:86-109)."""
        for name, q in (rl or {}).items():
            if name == CPU:
                self.cpu += q_milli(q)
            elif name == MEM:
                self.mem += q_value(q)
            elif name == GPU:
                self.gpu += q_value(q)
            elif name == PODS:
                self.pods += q_value(q)
            elif name == EPH:
                self.eph += q_value(q)
            elif is_scalar_resource_name(name):
                self.scalar[name] = self.scalar.get(name, 0) + q_value(q)


def _containers(pod, key="containers"):
    return (pod.get("spec") or {}).get(key) or []


def _requests(c):
    return ((c.get("resources") or {}).get("requests")) or {}


def _limits(c):
    return ((c.get("resources") or {}).get("limits")) or {}


def get_resource_request(pod) -> Resource:
    """predicates.go:659-697: sum of containers, max'd with each init container."""
    r = Resource()
    for c in _containers(pod):
        r.add(_requests(c))
    for c in _containers(pod, "initContainers"):
        for name, q in _requests(c).items():
            if name == MEM:
                r.mem = max(r.mem, q_value(q))
            elif name == EPH:
                r.eph = max(r.eph, q_value(q))
            elif name == CPU:
                r.cpu = max(r.cpu, q_milli(q))
            elif name == GPU:
                r.gpu = max(r.gpu, q_value(q))
            elif is_scalar_resource_name(name):
                v = q_value(q)
                if v > r.scalar.get(name, 0):
                    r.scalar[name] = v
    return r


DEFAULT_MILLI_CPU = 100                 # priorities/util/non_zero.go:31
DEFAULT_MEMORY = 200 * 1024 * 1024      # priorities/util/non_zero.go:33


def nonzero_requests(reqs: dict):
    """GetNonzeroRequests (priorities/util/non_zero.go:38-53)."""
    cpu = DEFAULT_MILLI_CPU if CPU not in reqs else q_milli(reqs[CPU])
    mem = DEFAULT_MEMORY if MEM not in reqs else q_value(reqs[MEM])
    return cpu, mem


def calculate_resource(pod):
    """node_info.go:400-412: containers only; returns (Resource, nzcpu, nzmem)."""
    r = Resource()
    nzc = nzm = 0
    for c in _containers(pod):
        r.add(_requests(c))
        a, b = nonzero_requests(_requests(c))
        nzc += a
        nzm += b
    return r, nzc, nzm


def get_nonzero_pod(pod):
    """priorities/resource_allocation.go:76-85."""
    nzc = nzm = 0
    for c in _containers(pod):
        a, b = nonzero_requests(_requests(c))
        nzc += a
        nzm += b
    return nzc, nzm


def is_best_effort(pod) -> bool:
    """K/pkg/apis/core/v1/helper/qos/qos.go:39-85 (BestEffort iff no positive
    cpu/memory request or limit in any container)."""
    for c in _containers(pod):
        for rl in (_requests(c), _limits(c)):
            for name, q in rl.items():
                if name in (CPU, MEM) and parse_quantity(q) > 0:
                    return False
    return True


# --------------------------------------------------------------------------
# Host ports (S/util/utils.go:31-155)
# --------------------------------------------------------------------------
def _sanitize(ip, proto):
    return (ip or "0.0.0.0"), (proto or "TCP")


def pod_ports(pod):
    """GetContainerPorts (S/util/utils.go:144-155)."""
    out = []
    for c in _containers(pod):
        for p in c.get("ports") or []:
            out.append((p.get("hostIP", ""), p.get("protocol", ""), int(p.get("hostPort", 0) or 0)))
    return out


def check_conflict(used: set, ip, proto, port) -> bool:
    """HostPortInfo.CheckConflict (S/util/utils.go:101-130)."""
    if port <= 0:
        return False
    ip, proto = _sanitize(ip, proto)
    if ip == "0.0.0.0":
        return any((p == proto and n == port) for (_i, p, n) in used)
    return ("0.0.0.0", proto, port) in used or (ip, proto, port) in used


# --------------------------------------------------------------------------
# Labels (AM/pkg/labels/selector.go)
# --------------------------------------------------------------------------
_QN_NAME = re.compile(r"^([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]$")
_DNS1123_SUB = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*$")
_LABEL_VALUE = re.compile(r"^(([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])?$")


def valid_label_key(k: str) -> bool:
    """validateLabelKey → IsQualifiedName (apimachinery/pkg/util/validation)."""
    parts = k.split("/")
    if len(parts) == 1:
        name = parts[0]
    elif len(parts) == 2:
        prefix, name = parts
        if len(prefix) == 0 or len(prefix) > 253 or not _DNS1123_SUB.match(prefix):
            return False
    else:
        return False
    return 0 < len(name) <= 63 and bool(_QN_NAME.match(name))


def valid_label_value(v: str) -> bool:
    return len(v) <= 63 and bool(_LABEL_VALUE.match(v))


class Requirement:
    """labels.Requirement (selector.go:130-235)."""

    def __init__(self, key, op, values):
        self.key, self.op, self.values = key, op, list(values)

    def matches(self, labels: dict) -> bool:
        op = self.op
        if op in ("In", "=", "=="):
            return self.key in labels and labels[self.key] in self.values
        if op in ("NotIn", "!="):
            return self.key not in labels or labels[self.key] not in self.values
        if op == "Exists":
            return self.key in labels
        if op == "DoesNotExist":
            return self.key not in labels
        if op in ("Gt", "Lt"):
            if self.key not in labels:
                return False
            try:
                lv = _parse_int64(labels[self.key])
            except ValueError:
                return False
            if len(self.values) != 1:
                return False
            rv = _parse_int64(self.values[0])
            return (op == "Gt" and lv > rv) or (op == "Lt" and lv < rv)
        return False


def _parse_int64(s: str) -> int:
    """strconv.ParseInt(s, 10, 64)."""
    if not re.fullmatch(r"[+-]?[0-9]+", s):
        raise ValueError(s)
    v = int(s)
    if v < -(2 ** 63) or v > 2 ** 63 - 1:
        raise ValueError(s)
    return v


def new_requirement(key, op, vals):
    """NewRequirement validation (selector.go:130-178); raises on error."""
    if not valid_label_key(key):
        raise ValueError("bad key")
    if op in ("In", "NotIn"):
        if len(vals) == 0:
            raise ValueError("empty values")
    elif op in ("=", "==", "!="):
        if len(vals) != 1:
            raise ValueError("one value")
    elif op in ("Exists", "DoesNotExist"):
        if len(vals) != 0:
            raise ValueError("no values")
    elif op in ("Gt", "Lt"):
        if len(vals) != 1:
            raise ValueError("one value")
        _parse_int64(vals[0])
    else:
        raise ValueError("bad op")
    for v in vals:
        if not valid_label_value(v):
            raise ValueError("bad value")
    return Requirement(key, op, sorted(vals))


def selector_from_set(s: dict):
    """SelectorFromSet (selector.go:837-853): invalid entry → Everything()."""
    reqs = []
    for k, v in (s or {}).items():
        try:
            reqs.append(new_requirement(k, "=", [v]))
        except ValueError:
            return []
    return reqs


def selector_matches(reqs, labels) -> bool:
    return all(r.matches(labels) for r in reqs)


def node_selector_requirements_as_selector(exprs):
    """K/pkg/apis/core/v1/helper/helpers.go:215-245. Returns None for Nothing()."""
    if not exprs:
        return None
    reqs = []
    for e in exprs:
        op = e.get("operator")
        if op not in ("In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt"):
            raise ValueError("bad operator")
        reqs.append(new_requirement(e.get("key", ""), op, e.get("values") or []))
    return reqs


def node_matches_terms(labels, terms) -> bool:
    """predicates.go:780-793 nodeMatchesNodeSelectorTerms."""
    for t in terms or []:
        try:
            sel = node_selector_requirements_as_selector(t.get("matchExpressions") or [])
        except ValueError:
            return False
        if sel is not None and selector_matches(sel, labels):
            return True
    return False


def pod_matches_node_labels(pod, node) -> bool:
    """predicates.go:795-838."""
    spec = pod.get("spec") or {}
    labels = (node.get("metadata") or {}).get("labels") or {}
    ns = spec.get("nodeSelector") or {}
    if len(ns) > 0:
        if not selector_matches(selector_from_set(ns), labels):
            return False
    aff = spec.get("affinity") or {}
    na = aff.get("nodeAffinity")
    if na is not None:
        req = na.get("requiredDuringSchedulingIgnoredDuringExecution")
        if req is None:
            return True
        return node_matches_terms(labels, req.get("nodeSelectorTerms") or [])
    return True


# --------------------------------------------------------------------------
# Taints / tolerations (vendor/k8s.io/api/core/v1/toleration.go:37-56,
# K/pkg/apis/core/v1/helper/helpers.go:282-313)
# --------------------------------------------------------------------------
def tolerates_taint(tol, taint) -> bool:
    eff = tol.get("effect", "")
    if eff and eff != taint.get("effect", ""):
        return False
    key = tol.get("key", "")
    if key and key != taint.get("key", ""):
        return False
    op = tol.get("operator", "")
    if op in ("", "Equal"):
        return tol.get("value", "") == taint.get("value", "")
    if op == "Exists":
        return True
    return False


def tolerations_tolerate_taint(tols, taint) -> bool:
    return any(tolerates_taint(t, taint) for t in tols)


def tolerations_tolerate_taints_with_filter(tols, taints, filt) -> bool:
    for t in taints or []:
        if filt is not None and not filt(t):
            continue
        if not tolerations_tolerate_taint(tols, t):
            return False
    return True


# --------------------------------------------------------------------------
# NodeInfo (S/schedulercache/node_info.go)
# --------------------------------------------------------------------------
class NodeInfo:
    def __init__(self, node=None):
        self.node = None
        self.pods = []
        self.pods_with_affinity = []     # PodsWithAffinity (node_info.go:326-328)
        self.requested = Resource()
        self.nonzero_cpu = 0
        self.nonzero_mem = 0
        self.allocatable = Resource()
        self.used_ports = set()
        self.taints = []
        self.mem_pressure = ""
        self.disk_pressure = ""
        if node is not None:
            self.set_node(node)

    @property
    def name(self):
        return (self.node.get("metadata") or {}).get("name", "") if self.node else ""

    def set_node(self, node):
        """SetNode (node_info.go:429-448)."""
        self.node = node
        self.allocatable = Resource()
        self.allocatable.add((node.get("status") or {}).get("allocatable") or {})
        self.taints = (node.get("spec") or {}).get("taints") or []
        for c in (node.get("status") or {}).get("conditions") or []:
            if c.get("type") == "MemoryPressure":
                self.mem_pressure = c.get("status", "")
            elif c.get("type") == "DiskPressure":
                self.disk_pressure = c.get("status", "")

    def add_pod(self, pod):
        """AddPod (node_info.go:318-341)."""
        res, nzc, nzm = calculate_resource(pod)
        self.requested.cpu += res.cpu
        self.requested.mem += res.mem
        self.requested.gpu += res.gpu
        self.requested.eph += res.eph
        for k, v in res.scalar.items():
            self.requested.scalar[k] = self.requested.scalar.get(k, 0) + v
        self.nonzero_cpu += nzc
        self.nonzero_mem += nzm
        self.pods.append(pod)
        if has_pod_affinity_constraints(pod):
            self.pods_with_affinity.append(pod)
        for ip, proto, port in pod_ports(pod):
            if port > 0:
                self.used_ports.add(_sanitize(ip, proto) + (port,))

    def remove_pod(self, pod):
        """RemovePod (node_info.go:343-390): the containers-only requests come off, the pod's
        ports leave the HostPortInfo set (utils.go:63-79 Remove deletes the key)."""
        key = pod_key(pod)
        for i, p in enumerate(self.pods):
            if pod_key(p) != key:
                continue
            self.pods[i] = self.pods[-1]
            self.pods.pop()
            for j, q in enumerate(self.pods_with_affinity):
                if pod_key(q) == key:
                    del self.pods_with_affinity[j]
                    break
            res, nzc, nzm = calculate_resource(pod)
            self.requested.cpu -= res.cpu
            self.requested.mem -= res.mem
            self.requested.gpu -= res.gpu
            self.requested.eph -= res.eph
            for k, v in res.scalar.items():
                self.requested.scalar[k] = self.requested.scalar.get(k, 0) - v
            self.nonzero_cpu -= nzc
            self.nonzero_mem -= nzm
            for ip, proto, port in pod_ports(pod):
                if port > 0:
                    self.used_ports.discard(_sanitize(ip, proto) + (port,))
            return
        raise KeyError("no corresponding pod %s in pods of node %s" % ((pod.get("metadata") or {}).get("name"), self.name))

    def remove_node(self):
        """RemoveNode (node_info.go:450-463)."""
        self.node = None
        self.allocatable = Resource()
        self.taints = []
        self.mem_pressure = "Unknown"
        self.disk_pressure = "Unknown"


def pod_key(pod):
    """getPodKey (node_info.go:497-503) is the UID; pods without one are keyed by namespace/name."""
    md = pod.get("metadata") or {}
    return md.get("uid") or "%s/%s" % (md.get("namespace", ""), md.get("name", ""))


# --------------------------------------------------------------------------
# Predicates (S/algorithm/predicates/predicates.go)
# --------------------------------------------------------------------------
R_NOT_READY = "node(s) were not ready"
R_OUT_OF_DISK = "node(s) were out of disk space"
R_NET_UNAVAIL = "node(s) had unavailable network"
R_UNSCHED = "node(s) were unschedulable"
R_HOSTNAME = "node(s) didn't match the requested hostname"
R_PORTS = "node(s) didn't have free ports for the requested pod ports"
R_SELECTOR = "node(s) didn't match node selector"
R_TAINTS = "node(s) had taints that the pod didn't tolerate"
R_MEM_PRESSURE = "node(s) had memory pressure"
R_DISK_PRESSURE = "node(s) had disk pressure"


def insufficient(name):
    return "Insufficient " + name


def pred_check_node_condition(pod, ni):
    """predicates.go:1534-1568."""
    reasons = []
    node = ni.node
    for c in (node.get("status") or {}).get("conditions") or []:
        t, s = c.get("type"), c.get("status")
        if t == "Ready" and s != "True":
            reasons.append(R_NOT_READY)
        elif t == "OutOfDisk" and s != "False":
            reasons.append(R_OUT_OF_DISK)
        elif t == "NetworkUnavailable" and s != "False":
            reasons.append(R_NET_UNAVAIL)
    if (node.get("spec") or {}).get("unschedulable"):
        reasons.append(R_UNSCHED)
    return not reasons, reasons


def pred_check_node_unschedulable(pod, ni):
    """predicates.go CheckNodeUnschedulablePredicate."""
    if (ni.node.get("spec") or {}).get("unschedulable"):
        return False, [R_UNSCHED]
    return True, []


def pred_pod_fits_resources(pod, ni):
    """predicates.go:706-778."""
    fails = []
    allowed = ni.allocatable.pods
    if len(ni.pods) + 1 > allowed:
        fails.append(insufficient(PODS))
    req = get_resource_request(pod)
    if req.cpu == 0 and req.mem == 0 and req.gpu == 0 and req.eph == 0 and len(req.scalar) == 0:
        return not fails, fails
    a, r = ni.allocatable, ni.requested
    if a.cpu < req.cpu + r.cpu:
        fails.append(insufficient(CPU))
    if a.mem < req.mem + r.mem:
        fails.append(insufficient(MEM))
    if a.gpu < req.gpu + r.gpu:
        fails.append(insufficient(GPU))
    if a.eph < req.eph + r.eph:
        fails.append(insufficient(EPH))
    for name in sorted(req.scalar):
        if a.scalar.get(name, 0) < req.scalar[name] + r.scalar.get(name, 0):
            fails.append(insufficient(name))
    return not fails, fails


def pred_pod_fits_host(pod, ni):
    """predicates.go:853-866."""
    nn = (pod.get("spec") or {}).get("nodeName", "")
    if not nn:
        return True, []
    if nn == ni.name:
        return True, []
    return False, [R_HOSTNAME]


def pred_pod_fits_host_ports(pod, ni):
    """predicates.go:1019-1039 + utils.go:138-148."""
    want = pod_ports(pod)
    if not want:
        return True, []
    for ip, proto, port in want:
        if check_conflict(ni.used_ports, ip, proto, port):
            return False, [R_PORTS]
    return True, []


def pred_match_node_selector(pod, ni):
    """predicates.go:841-850."""
    if pod_matches_node_labels(pod, ni.node):
        return True, []
    return False, [R_SELECTOR]


def pred_general(pod, ni):
    """predicates.go:1059-1120: resources, then host, ports, selector; no short-circuit."""
    fails = []
    for f in (pred_pod_fits_resources, pred_pod_fits_host, pred_pod_fits_host_ports, pred_match_node_selector):
        ok, rs = f(pod, ni)
        if not ok:
            fails.extend(rs)
    return not fails, fails


def pred_tolerates_taints(pod, ni):
    """predicates.go:1465-1474."""
    tols = (pod.get("spec") or {}).get("tolerations") or []
    if tolerations_tolerate_taints_with_filter(tols, ni.taints, lambda t: t.get("effect") in ("NoSchedule", "NoExecute")):
        return True, []
    return False, [R_TAINTS]


def pred_tolerates_noexec_taints(pod, ni):
    tols = (pod.get("spec") or {}).get("tolerations") or []
    if tolerations_tolerate_taints_with_filter(tols, ni.taints, lambda t: t.get("effect") == "NoExecute"):
        return True, []
    return False, [R_TAINTS]


def pred_memory_pressure(pod, ni):
    """predicates.go:1502-1521."""
    if not is_best_effort(pod):
        return True, []
    if ni.mem_pressure == "True":
        return False, [R_MEM_PRESSURE]
    return True, []


def pred_disk_pressure(pod, ni):
    """predicates.go:1524-1530."""
    if ni.disk_pressure == "True":
        return False, [R_DISK_PRESSURE]
    return True, []


def pred_true(pod, ni):
    return True, []


# --------------------------------------------------------------------------
# Volume predicates (predicates.go:205-633)
# --------------------------------------------------------------------------
R_DISK_CONFLICT = "node(s) had no available disk"                  # error.go:35
R_MAX_VOLUME_COUNT = "node(s) exceed max volume count"             # error.go:59
R_VOLUME_ZONE = "node(s) had no available volume zone"             # error.go:37
ZONE_LABEL = "failure-domain.beta.kubernetes.io/zone"              # kubelet/apis/well_known_labels.go:21
REGION_LABEL = "failure-domain.beta.kubernetes.io/region"          # :23
DEFAULT_MAX_VOLS = {"EBS": 39, "GCE": 16, "AzureDisk": 16}          # predicates.go:93-103


class PredicateError(Exception):
    """A predicate's error return (not a failure reason): findNodesThatFit aborts the pod's
    scheduling cycle with it (core/generic_scheduler.go:351-353)."""


def _src(vol, kind):
    """The VolumeSource member `kind` (nil when absent, generic_scheduler's != nil tests)."""
    return vol.get(kind)


def _volumes(pod):
    return (pod.get("spec") or {}).get("volumes") or []


def have_overlap(a1, a2):
    """predicates.go:1042-1055."""
    m = set(a1 or [])
    return any(v in m for v in a2 or [])


def is_volume_conflict(volume, pod):
    """isVolumeConflict (predicates.go:220-265): `volume` of the incoming pod against every
    volume of an existing pod."""
    gce, ebs = _src(volume, "gcePersistentDisk"), _src(volume, "awsElasticBlockStore")
    rbd, iscsi = _src(volume, "rbd"), _src(volume, "iscsi")
    if gce is None and ebs is None and rbd is None and iscsi is None:
        return False
    for ev in _volumes(pod):
        egce = _src(ev, "gcePersistentDisk")
        if gce is not None and egce is not None:
            if gce.get("pdName", "") == egce.get("pdName", "") and not (gce.get("readOnly") and egce.get("readOnly")):
                return True
        eebs = _src(ev, "awsElasticBlockStore")
        if ebs is not None and eebs is not None:
            if ebs.get("volumeID", "") == eebs.get("volumeID", ""):
                return True
        eis = _src(ev, "iscsi")
        if iscsi is not None and eis is not None:
            if iscsi.get("iqn", "") == eis.get("iqn", "") and not (iscsi.get("readOnly") and eis.get("readOnly")):
                return True
        erbd = _src(ev, "rbd")
        if rbd is not None and erbd is not None:
            if (have_overlap(rbd.get("monitors"), erbd.get("monitors")) and rbd.get("pool", "") == erbd.get("pool", "")
                    and rbd.get("image", "") == erbd.get("image", "")
                    and not (rbd.get("readOnly") and erbd.get("readOnly"))):
                return True
    return False


def pred_no_disk_conflict(pod, ni):
    """NoDiskConflict (predicates.go:276-285)."""
    for v in _volumes(pod):
        for ev in ni.pods:
            if is_volume_conflict(v, ev):
                return False, [R_DISK_CONFLICT]
    return True, []


def go_atoi(s):
    """strconv.Atoi: optional sign, decimal digits, int64 range; None on error."""
    import re as _re
    if not _re.fullmatch(r"[+-]?[0-9]+", s or ""):
        return None
    v = int(s)
    return v if -(1 << 63) <= v < (1 << 63) else None


def get_max_vols(default, raw=None):
    """getMaxVols (predicates.go:347-359): KUBE_MAX_PD_VOLS when it parses to a positive int."""
    if raw is None:
        raw = os.environ.get("KUBE_MAX_PD_VOLS", "")
    if raw != "":
        v = go_atoi(raw)
        if v is not None and v > 0:
            return v
    return default


# VolumeFilter.FilterVolume / FilterPersistentVolume (predicates.go:458-507): (source key, id field)
VOLUME_FILTERS = {"EBS": ("awsElasticBlockStore", "volumeID"), "GCE": ("gcePersistentDisk", "pdName"),
                  "AzureDisk": ("azureDisk", "diskName")}


class VolumeListers:
    """PersistentVolumeInfo / PersistentVolumeClaimInfo: the simulator's PV / PVC informers are
    empty (its store only ever holds nodes and pods, pkg/main.go:147-179), so by default every
    lookup misses; tests pass the reference tests' fake listers (testing_helper.go:30-72)."""

    def __init__(self, pvs=(), pvcs=(), classes=()):
        self.pvs = {(x.get("metadata") or {}).get("name", ""): x for x in pvs}
        self.pvcs = {((x.get("metadata") or {}).get("namespace", ""), (x.get("metadata") or {}).get("name", "")): x
                     for x in pvcs}
        self.classes = {(x.get("metadata") or {}).get("name", ""): x for x in classes}

    def pvc(self, ns, name):
        return self.pvcs.get((ns, name))

    def pv(self, name):
        return self.pvs.get(name)


PV_ID_PREFIX = "ksim-random-prefix"   # rand.String(32) in the reference; any value no real id uses


class MaxPDVolumeCountChecker:
    """MaxPDVolumeCountChecker (predicates.go:287-456)."""

    def __init__(self, filter_name, listers=None, max_vols=None):
        self.kind, self.field = VOLUME_FILTERS[filter_name]
        self.max_vols = get_max_vols(DEFAULT_MAX_VOLS[filter_name]) if max_vols is None else max_vols
        self.listers = listers or VolumeListers()

    def _filter(self, src):
        s = src.get(self.kind)
        return (s.get(self.field, ""), True) if s is not None else ("", False)

    def filter_volumes(self, volumes, namespace, out):
        """filterVolumes (:361-413)."""
        for vol in volumes:
            vid, ok = self._filter(vol)
            if ok:
                out.add(vid)
                continue
            claim = vol.get("persistentVolumeClaim")
            if claim is None:
                continue
            name = claim.get("claimName", "")
            if name == "":
                raise PredicateError("PersistentVolumeClaim had no name")
            pv_id = "%s-%s/%s" % (PV_ID_PREFIX, namespace, name)
            pvc = self.listers.pvc(namespace, name)
            if pvc is None:
                out.add(pv_id)
                continue
            pv_name = (pvc.get("spec") or {}).get("volumeName", "")
            if pv_name == "":
                out.add(pv_id)
                continue
            pv = self.listers.pv(pv_name)
            if pv is None:
                out.add(pv_id)
                continue
            vid, ok = self._filter(pv.get("spec") or {})
            if ok:
                out.add(vid)

    def predicate(self, pod, ni):
        """predicate (:415-456)."""
        vols = _volumes(pod)
        if not vols:
            return True, []
        new = set()
        self.filter_volumes(vols, (pod.get("metadata") or {}).get("namespace", ""), new)
        if not new:
            return True, []
        existing = set()
        for ep in ni.pods:
            self.filter_volumes(_volumes(ep), (ep.get("metadata") or {}).get("namespace", ""), existing)
        if len(existing) + len(new - existing) > self.max_vols:
            return False, [R_MAX_VOLUME_COUNT]
        return True, []


def label_zones_to_set(v):
    """volumeutil.LabelZonesToSet (pkg/volume/util/util.go:357-376); None on a parse error."""
    out = set()
    for z in v.split("__"):
        t = z.strip(" \t\n\r\v\f")
        if t == "":
            return None
        out.add(t)
    return out


def new_volume_zone_predicate(listers=None, volume_scheduling=True):
    """VolumeZoneChecker.predicate (predicates.go:539-633).  volume_scheduling: the
    VolumeScheduling feature gate (beta, on by default in v1.10: kube_features.go:309)."""
    listers = listers or VolumeListers()

    def pred(pod, ni):
        vols = _volumes(pod)
        if not vols:
            return True, []
        node = ni.node
        if node is None:
            raise PredicateError("node not found")
        cons = {k: v for k, v in ((node.get("metadata") or {}).get("labels") or {}).items()
                if k in (ZONE_LABEL, REGION_LABEL)}
        if not cons:
            return True, []
        ns = (pod.get("metadata") or {}).get("namespace", "")
        for vol in vols:
            claim = vol.get("persistentVolumeClaim")
            if claim is None:
                continue
            name = claim.get("claimName", "")
            if name == "":
                raise PredicateError("PersistentVolumeClaim had no name")
            pvc = listers.pvc(ns, name)
            if pvc is None:
                raise PredicateError("persistentvolumeclaim %r not found" % name)
            pv_name = (pvc.get("spec") or {}).get("volumeName", "")
            if pv_name == "":
                if volume_scheduling:
                    sc = (pvc.get("spec") or {}).get("storageClassName")
                    if sc:
                        cls = listers.classes.get(sc)
                        if cls is not None:
                            mode = cls.get("volumeBindingMode")
                            if mode is None:
                                raise PredicateError("VolumeBindingMode not set for StorageClass %r" % sc)
                            if mode == "WaitForFirstConsumer":
                                continue
                raise PredicateError("PersistentVolumeClaim is not bound: %r" % name)
            pv = listers.pv(pv_name)
            if pv is None:
                raise PredicateError("PersistentVolume not found: %r" % pv_name)
            for k, v in ((pv.get("metadata") or {}).get("labels") or {}).items():
                if k not in (ZONE_LABEL, REGION_LABEL):
                    continue
                zones = label_zones_to_set(v)
                if zones is None:
                    continue   # unparsable label: ignored (:619-622)
                if cons.get(k, "") not in zones:
                    return False, [R_VOLUME_ZONE]
        return True, []
    return pred


def new_volume_binding_predicate(listers=None):
    """VolumeBindingChecker.predicate (predicates.go:1586-1618) with the VolumeScheduling gate on:
    FindPodVolumes (scheduler_binder.go:127-167, getPodVolumes :290-320).  A PVC the listers do not
    hold, or an unbound one without a WaitForFirstConsumer class, is an error; a bound PVC checks
    its PV's node affinity, which only PVs without one satisfy here (others: PredicateError, the
    outside-the-supported-set marker)."""
    listers = listers or VolumeListers()

    def pred(pod, ni):
        if ni.node is None:
            raise PredicateError("node not found")
        ns = (pod.get("metadata") or {}).get("namespace", "")
        for vol in _volumes(pod):
            claim = vol.get("persistentVolumeClaim")
            if claim is None:
                continue
            pvc = listers.pvc(ns, claim.get("claimName", ""))
            if pvc is None:
                raise PredicateError("error getting PVC %r" % claim.get("claimName", ""))
            pv = listers.pv((pvc.get("spec") or {}).get("volumeName", ""))
            if pv is None or (pv.get("spec") or {}).get("nodeAffinity") is not None:
                raise PredicateError("volume binding outside the restated cases")
        return True, []
    return pred


def volume_predicates(listers=None, max_vols=None):
    """The volume predicates over `listers`, by key (custom_predicates form); max_vols: a
    KUBE_MAX_PD_VOLS value (None: the environment's)."""
    out = {"NoDiskConflict": pred_no_disk_conflict,
           "NoVolumeZoneConflict": new_volume_zone_predicate(listers),
           "CheckVolumeBinding": new_volume_binding_predicate(listers)}
    for key, f in (("MaxEBSVolumeCount", "EBS"), ("MaxGCEPDVolumeCount", "GCE"),
                   ("MaxAzureDiskVolumeCount", "AzureDisk")):
        mv = None if max_vols is None else get_max_vols(DEFAULT_MAX_VOLS[f], str(max_vols))
        out[key] = MaxPDVolumeCountChecker(f, listers, mv).predicate
    return out


PREDICATES = {
    "CheckNodeCondition": pred_check_node_condition,
    "CheckNodeUnschedulable": pred_check_node_unschedulable,
    "GeneralPredicates": pred_general,
    "HostName": pred_pod_fits_host,
    "PodFitsHostPorts": pred_pod_fits_host_ports,
    "PodFitsPorts": pred_pod_fits_host_ports,
    "MatchNodeSelector": pred_match_node_selector,
    "PodFitsResources": pred_pod_fits_resources,
    "NoDiskConflict": pred_no_disk_conflict,
    "PodToleratesNodeTaints": pred_tolerates_taints,
    "PodToleratesNodeNoExecuteTaints": pred_tolerates_noexec_taints,
    # the simulator's (empty) PV / PVC listers; volume_predicates() builds them over others
    "MaxEBSVolumeCount": MaxPDVolumeCountChecker("EBS").predicate,
    "MaxGCEPDVolumeCount": MaxPDVolumeCountChecker("GCE").predicate,
    "MaxAzureDiskVolumeCount": MaxPDVolumeCountChecker("AzureDisk").predicate,
    "CheckVolumeBinding": new_volume_binding_predicate(),
    "NoVolumeZoneConflict": new_volume_zone_predicate(),
    "CheckNodeMemoryPressure": pred_memory_pressure,
    "CheckNodeDiskPressure": pred_disk_pressure,
    "MatchInterPodAffinity": pred_true,   # replaced per scheduling cycle (GenericScheduler.schedule)
}

# predicates.go:129-138 (PodFitsPorts is registered under its own key but is not
# in the ordering list, so it never runs from podFitsOnNode)
ORDERING = ["CheckNodeCondition", "CheckNodeUnschedulable", "GeneralPredicates", "HostName",
            "PodFitsHostPorts", "MatchNodeSelector", "PodFitsResources", "NoDiskConflict",
            "PodToleratesNodeTaints", "PodToleratesNodeNoExecuteTaints", "CheckNodeLabelPresence",
            "CheckServiceAffinity", "MaxEBSVolumeCount", "MaxGCEPDVolumeCount",
            "MaxAzureDiskVolumeCount", "CheckVolumeBinding", "NoVolumeZoneConflict",
            "CheckNodeMemoryPressure", "CheckNodeDiskPressure", "MatchInterPodAffinity"]


R_SERVICE_AFFINITY = "node(s) didn't match service affinity"   # error.go:57


def new_service_affinity_predicate(affinity_labels, services=(), pods=(), nodes=()):
    """ServiceAffinity.checkServiceAffinity (predicates.go:940-1016) with its metadata producer
    (:958-978): `services` what the ServiceLister holds, `pods` the PodLister's pods (in its order),
    `nodes` the NodeLister's nodes.  The node must carry the pod's nodeSelector values of the listed
    labels; when some are missing and a service selects the pod, the first pod with the pod's
    labels (FilterOutPods, node_info.go:466-488) lends its node's values."""
    by_name = {(n.get("metadata") or {}).get("name", ""): n for n in nodes}

    def pred(pod, ni):
        md = pod.get("metadata") or {}
        ns, lab = md.get("namespace", ""), md.get("labels") or {}
        svcs = [x for x in services if (x.get("metadata") or {}).get("namespace", "") == ns and
                (x.get("spec") or {}).get("selector") is not None and
                SpreadListers._set_matches((x.get("spec") or {}).get("selector"), lab)]
        own = selector_from_set(lab)
        matching = [q for q in pods if (q.get("metadata") or {}).get("namespace", "") == ns and
                    selector_matches(own, (q.get("metadata") or {}).get("labels") or {})]
        keys = {pod_key(q) for q in ni.pods}
        filtered = [q for q in matching
                    if (q.get("spec") or {}).get("nodeName", "") != ni.name or pod_key(q) in keys]
        sel = (pod.get("spec") or {}).get("nodeSelector") or {}
        al = {k: sel[k] for k in affinity_labels if k in sel}
        if len(affinity_labels) > len(al) and svcs and filtered:
            nn = (filtered[0].get("spec") or {}).get("nodeName", "")
            if nn not in by_name:
                raise PredicateError("node %r not found" % nn)
            nl = (by_name[nn].get("metadata") or {}).get("labels") or {}
            for k in affinity_labels:
                if k not in al and k in nl:
                    al[k] = nl[k]
        node_labels = (ni.node.get("metadata") or {}).get("labels") or {}
        if selector_matches(selector_from_set(al), node_labels):
            return True, []
        return False, [R_SERVICE_AFFINITY]
    return pred


R_LABEL_PRESENCE = "node(s) didn't have the requested labels"


def new_node_label_predicate(labels, presence):
    """NewNodeLabelPredicate / CheckNodeLabelPresence (predicates.go:875-910): every listed
    label present (presence=True) or absent (False), values ignored."""
    def pred(pod, ni):
        node_labels = (ni.node.get("metadata") or {}).get("labels") or {}
        for label in labels:
            if (label in node_labels) != presence:
                return False, [R_LABEL_PRESENCE]
        return True, []
    return pred


# --------------------------------------------------------------------------
# Inter-pod affinity: the MatchInterPodAffinity predicate (S/algorithm/predicates/
# predicates.go:1143-1450, metadata S/algorithm/predicates/metadata.go:102-123) and
# InterPodAffinityPriority (S/algorithm/priorities/interpod_affinity.go:118-240), with the
# helpers of S/algorithm/priorities/util/topologies.go:28-71 and
# AM/pkg/apis/meta/v1/helpers.go LabelSelectorAsSelector.
# --------------------------------------------------------------------------
HOSTNAME_LABEL = "kubernetes.io/hostname"     # kubeletapis.LabelHostname
R_AFFINITY = "node(s) didn't match pod affinity/anti-affinity"
R_AFFINITY_RULES = "node(s) didn't match pod affinity rules"
R_ANTI_AFFINITY_RULES = "node(s) didn't match pod anti-affinity rules"
R_EXISTING_ANTI = "node(s) didn't satisfy existing pods anti-affinity rules"
NOTHING = None                                 # labels.Nothing(): matches no pod


class AffinityError(Exception):
    """An error the reference returns (not a FitError): bad selector, empty topologyKey on a
    required term, an existing pod's node missing from the node lister."""


def label_selector_as_selector(ps):
    """metav1.LabelSelectorAsSelector: nil → Nothing, empty → Everything ([]), else the
    requirements (matchLabels as Equals, matchExpressions In/NotIn/Exists/DoesNotExist)."""
    if ps is None:
        return NOTHING
    ml, me = ps.get("matchLabels") or {}, ps.get("matchExpressions") or []
    if not ml and not me:
        return []
    reqs = []
    try:
        for k in sorted(ml):
            reqs.append(new_requirement(k, "=", [ml[k]]))
        for e in me:
            op = e.get("operator")
            if op not in ("In", "NotIn", "Exists", "DoesNotExist"):
                raise AffinityError("%r is not a valid pod selector operator" % op)
            reqs.append(new_requirement(e.get("key", ""), op, list(e.get("values") or [])))
    except ValueError as err:
        raise AffinityError(str(err))
    return reqs


def _meta(obj):
    return obj.get("metadata") or {}


def term_namespaces(pod, term):
    """GetNamespacesFromPodAffinityTerm: the term's namespaces, or the defining pod's."""
    ns = term.get("namespaces") or []
    return set(ns) if ns else {_meta(pod).get("namespace", "")}


def pod_matches_term(pod, namespaces, sel):
    """PodMatchesTermsNamespaceAndSelector."""
    if _meta(pod).get("namespace", "") not in namespaces:
        return False
    if sel is NOTHING:
        return False
    return selector_matches(sel, _meta(pod).get("labels") or {})


def same_topology(node_a, node_b, key):
    """NodesHaveSameTopologyKey: both nodes carry label `key` with equal values."""
    if not key:
        return False
    la, lb = _meta(node_a).get("labels"), _meta(node_b).get("labels")
    if la is None or lb is None:
        return False
    return key in la and key in lb and la[key] == lb[key]


def _affinity(pod):
    return (pod.get("spec") or {}).get("affinity") or {}


def has_pod_affinity_constraints(pod):
    """hasPodAffinityConstraints (node_info.go): PodAffinity or PodAntiAffinity set."""
    a = _affinity(pod)
    return a.get("podAffinity") is not None or a.get("podAntiAffinity") is not None


def required_terms(section):
    """GetPodAffinityTerms / GetPodAntiAffinityTerms."""
    return list((section or {}).get("requiredDuringSchedulingIgnoredDuringExecution") or [])


def preferred_terms(section):
    return list((section or {}).get("preferredDuringSchedulingIgnoredDuringExecution") or [])


def matching_anti_affinity_terms(pod, pods_with_nodes):
    """getMatchingAntiAffinityTerms (predicates.go:1235-1293 over a nodeInfoMap's
    PodsWithAffinity, or the metadata-less :1313-1338 over the pod lister): every required
    anti-affinity term of an existing pod that `pod` matches, with the existing pod's node.
    pods_with_nodes: [(existing pod, its v1.Node)]."""
    out = []
    for e, enode in pods_with_nodes:
        if not has_pod_affinity_constraints(e):
            continue
        for t in required_terms(_affinity(e).get("podAntiAffinity")):
            sel = label_selector_as_selector(t.get("labelSelector"))
            if pod_matches_term(pod, term_namespaces(e, t), sel):
                out.append((t, enode))
    return out


def _any_pod_matches(pod, all_pods, node_pods, node, term):
    """anyPodMatchesPodAffinityTerm (predicates.go:1161-1194): (a matching pod on a node in the
    same topology, a matching pod anywhere); hostname terms only look at the node's own pods."""
    key = term.get("topologyKey", "")
    if not key:
        raise AffinityError("empty topologyKey is not allowed except for PreferredDuringScheduling pod anti-affinity")
    ns = term_namespaces(pod, term)
    sel = label_selector_as_selector(term.get("labelSelector"))
    pods = node_pods if key == HOSTNAME_LABEL else all_pods
    exists = False
    for e, enode in pods:
        if pod_matches_term(e, ns, sel):
            exists = True
            if same_topology(node, enode, key):
                return True, True
    return False, exists


def interpod_affinity_matches(pod, node, meta_terms, all_pods, node_pods):
    """PodAffinityChecker.InterPodAffinityMatches (predicates.go:1143-1156) → (fits, reasons,
    error) as Go returns them (an error comes with failure reasons; the scheduler turns it into
    a scheduling error, podFitsOnNode generic_scheduler.go:505-508).  node: the candidate
    v1.Node; meta_terms: matching_anti_affinity_terms of the predicate metadata; all_pods:
    podLister.FilteredList as [(pod, node)]; node_pods: nodeInfo.Pods() likewise."""
    for t, enode in meta_terms:          # satisfiesExistingPodsAntiAffinity (:1340-1379)
        if not t.get("topologyKey"):
            return False, [R_AFFINITY, R_EXISTING_ANTI], AffinityError("empty topologyKey")
        if same_topology(node, enode, t["topologyKey"]):
            return False, [R_AFFINITY, R_EXISTING_ANTI], None
    a = _affinity(pod)
    if a.get("podAffinity") is None and a.get("podAntiAffinity") is None:
        return True, [], None
    # satisfiesPodsAffinityAntiAffinity (:1382-1450)
    for t in required_terms(a.get("podAffinity")):
        try:
            matches, exists = _any_pod_matches(pod, all_pods, node_pods, node, t)
        except AffinityError as err:
            return False, [R_AFFINITY, R_AFFINITY_RULES], err
        if not matches:
            if exists:
                return False, [R_AFFINITY, R_AFFINITY_RULES], None
            try:
                sel = label_selector_as_selector(t.get("labelSelector"))
            except AffinityError as err:
                return False, [R_AFFINITY, R_AFFINITY_RULES], err
            if not pod_matches_term(pod, term_namespaces(pod, t), sel):
                return False, [R_AFFINITY, R_AFFINITY_RULES], None
    for t in required_terms(a.get("podAntiAffinity")):
        try:
            matches, _ = _any_pod_matches(pod, all_pods, node_pods, node, t)
        except AffinityError:
            matches = True               # the error is swallowed: the term fails (:1436-1441)
        if matches:
            return False, [R_AFFINITY, R_ANTI_AFFINITY_RULES], None
    return True, [], None


def _interpod_predicate(meta, all_pods):
    def pred(pod, ni):
        fits, reasons, err = interpod_affinity_matches(pod, ni.node, meta, all_pods, [(q, ni.node) for q in ni.pods])
        if err is not None:
            raise err
        return fits, reasons
    return pred


def interpod_affinity_priority(pod, infos, filtered_nodes, hard_weight):
    """CalculateInterPodAffinityPriority (interpod_affinity.go:118-240).  infos: the node infos
    of nodeNameToInfo (their pods; a pod's node is its info's node); filtered_nodes: the v1.Node
    list being prioritised.  Returns the 0..10 scores in filtered_nodes' order."""
    a = _affinity(pod)
    has_aff, has_anti = a.get("podAffinity") is not None, a.get("podAntiAffinity") is not None
    counts = [0.0] * len(filtered_nodes)

    def process_term(term, defining, to_check, fixed_node, weight):
        sel = label_selector_as_selector(term.get("labelSelector"))
        if pod_matches_term(to_check, term_namespaces(defining, term), sel):
            for k, n in enumerate(filtered_nodes):
                if same_topology(n, fixed_node, term.get("topologyKey", "")):
                    counts[k] += weight

    for info in infos:
        if info.node is None:
            continue
        pods = info.pods if (has_aff or has_anti) else info.pods_with_affinity
        if not pods:
            continue
        for e in pods:
            enode = info.node
            ea = _affinity(e)
            if has_aff:
                for wt in preferred_terms(a.get("podAffinity")):
                    process_term(wt.get("podAffinityTerm") or {}, pod, e, enode, float(wt.get("weight", 0)))
            if has_anti:
                for wt in preferred_terms(a.get("podAntiAffinity")):
                    process_term(wt.get("podAffinityTerm") or {}, pod, e, enode, float(-wt.get("weight", 0)))
            if ea.get("podAffinity") is not None:
                if hard_weight > 0:
                    for t in required_terms(ea.get("podAffinity")):
                        process_term(t, e, pod, enode, float(hard_weight))
                for wt in preferred_terms(ea.get("podAffinity")):
                    process_term(wt.get("podAffinityTerm") or {}, e, pod, enode, float(wt.get("weight", 0)))
            if ea.get("podAntiAffinity") is not None:
                for wt in preferred_terms(ea.get("podAntiAffinity")):
                    process_term(wt.get("podAffinityTerm") or {}, e, pod, enode, float(-wt.get("weight", 0)))
    mx = max([0.0] + counts)
    mn = min([0.0] + counts)
    out = []
    for c in counts:
        f = 0.0
        if mx - mn > 0:
            f = float(MAX_PRIORITY) * ((c - mn) / (mx - mn))
        out.append(int(f))
    return out


# factory/plugins.go:401-406 + defaults.go:165: always part of the predicate map
MANDATORY_PREDICATES = ("CheckNodeCondition",)


def pod_fits_on_node(pod, ni, keys, custom=None):
    """S/core/generic_scheduler.go:420-534 (nominated-pod pass inert; no ecache).  `custom`:
    predicates registered from a Policy argument (plugins.go:199-239), by key."""
    for k in ORDERING:
        if k in keys:
            fn = custom[k] if custom and k in custom else PREDICATES[k]
            ok, rs = fn(pod, ni)
            if not ok:
                return False, rs
    return True, []


# --------------------------------------------------------------------------
# Priorities (S/algorithm/priorities/*)
# --------------------------------------------------------------------------
MAX_PRIORITY = 10


def _least_score(req, cap):
    """least_requested.go:44-53 (Go int64 truncating division)."""
    if cap == 0 or req > cap:
        return 0
    return ((cap - req) * MAX_PRIORITY) // cap


def _most_score(req, cap):
    """most_requested.go:45-55."""
    if cap == 0 or req > cap:
        return 0
    return (req * MAX_PRIORITY) // cap


def _fraction(req, cap):
    """balanced_resource_allocation.go:57-61."""
    if cap == 0:
        return 1.0
    return float(req) / float(cap)


def _resource_requested(pod, ni):
    nzc, nzm = get_nonzero_pod(pod)
    return nzc + ni.nonzero_cpu, nzm + ni.nonzero_mem


def prio_least_requested(pod, ni):
    """resource_allocation.go:37-74 + least_requested.go:36-42."""
    c, m = _resource_requested(pod, ni)
    return (_least_score(c, ni.allocatable.cpu) + _least_score(m, ni.allocatable.mem)) // 2


def prio_most_requested(pod, ni):
    c, m = _resource_requested(pod, ni)
    return (_most_score(c, ni.allocatable.cpu) + _most_score(m, ni.allocatable.mem)) // 2


def prio_balanced(pod, ni):
    """balanced_resource_allocation.go:39-55 (IEEE doubles, trunc to int64)."""
    c, m = _resource_requested(pod, ni)
    fc = _fraction(c, ni.allocatable.cpu)
    fm = _fraction(m, ni.allocatable.mem)
    if fc >= 1 or fm >= 1:
        return 0
    diff = abs(fc - fm)
    return int((1 - diff) * float(MAX_PRIORITY))


def prio_taint_toleration_map(pod, ni):
    """taint_toleration.go:29-73."""
    tols = [t for t in ((pod.get("spec") or {}).get("tolerations") or [])
            if t.get("effect", "") in ("", "PreferNoSchedule")]
    cnt = 0
    for taint in ni.taints:
        if taint.get("effect") != "PreferNoSchedule":
            continue
        if not tolerations_tolerate_taint(tols, taint):
            cnt += 1
    return cnt


def prio_node_affinity_map(pod, ni):
    """node_affinity.go:34-75."""
    aff = ((pod.get("spec") or {}).get("affinity") or {}).get("nodeAffinity") or {}
    labels = (ni.node.get("metadata") or {}).get("labels") or {}
    count = 0
    for term in aff.get("preferredDuringSchedulingIgnoredDuringExecution") or []:
        w = int(term.get("weight", 0))
        if w == 0:
            continue
        sel = node_selector_requirements_as_selector((term.get("preference") or {}).get("matchExpressions") or [])
        if sel is not None and selector_matches(sel, labels):
            count += w
    return count


def normalize_reduce(scores, reverse):
    """reduce.go:29-64 (Go int truncating division)."""
    mx = 0
    for s in scores:
        if s > mx:
            mx = s
    if mx == 0:
        return [MAX_PRIORITY] * len(scores) if reverse else list(scores)
    out = []
    for s in scores:
        v = _go_div(MAX_PRIORITY * s, mx)
        out.append(MAX_PRIORITY - v if reverse else v)
    return out


def _go_div(a, b):
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def spread_reduce(scores, zones):
    """selector_spreading.go:121-174 with the map already computed."""
    counts_by_zone = {}
    max_node = 0
    for s, z in zip(scores, zones):
        if s > max_node:
            max_node = s
        if z == "":
            continue
        counts_by_zone[z] = counts_by_zone.get(z, 0) + s
    max_zone = 0
    for v in counts_by_zone.values():
        if v > max_zone:
            max_zone = v
    have_zones = len(counts_by_zone) != 0
    zw = 2.0 / 3.0
    out = []
    for s, z in zip(scores, zones):
        f = float(MAX_PRIORITY)
        if max_node > 0:
            f = float(MAX_PRIORITY) * (float(max_node - s) / float(max_node))
        if have_zones and z != "":
            zs = float(MAX_PRIORITY)
            if max_zone > 0:
                zs = float(MAX_PRIORITY) * (float(max_zone - counts_by_zone[z]) / float(max_zone))
            f = (f * (1.0 - zw)) + (zw * zs)
        out.append(int(f))
    return out


class SpreadListers:
    """ServiceLister / ControllerLister / ReplicaSetLister / StatefulSetLister as the scheduler's
    informer-backed listers answer (client-go listers core/v1/service_expansion.go:36-56,
    replicationcontroller_expansion.go:39-66, extensions/v1beta1/replicaset_expansion.go:41-73,
    apps/v1beta1/statefulset_expansion.go:41-80).  The simulator's are empty: its store holds no
    services and its controller informers are fake (pkg/scheduler/simulator.go:352-367)."""

    def __init__(self, services=(), rcs=(), rss=(), sss=()):
        self.services, self.rcs, self.rss, self.sss = list(services), list(rcs), list(rss), list(sss)

    @staticmethod
    def _set_matches(sel, lab):
        """labels.Set(sel).AsSelectorPreValidated().Matches."""
        return all(k in lab and lab[k] == v for k, v in sel.items())

    def selectors(self, pod, services_only=False):
        """getSelectors (priorities/metadata.go:82-114): the selectors of the services, RCs, RSs and
        StatefulSets selecting the pod (a lister error contributes nothing)."""
        md = pod.get("metadata") or {}
        ns, lab = md.get("namespace", ""), md.get("labels") or {}
        out = []
        for svc in self.services:
            sel = (svc.get("spec") or {}).get("selector")
            if (svc.get("metadata") or {}).get("namespace", "") != ns or sel is None:
                continue
            if self._set_matches(sel, lab):
                out.append(selector_from_set(sel))
        if services_only or not lab:
            return out            # the controller listers err for a pod without labels
        for rc in self.rcs:
            sel = (rc.get("spec") or {}).get("selector") or {}
            if (rc.get("metadata") or {}).get("namespace", "") == ns and sel and self._set_matches(sel, lab):
                out.append(selector_from_set(sel))
        for objs in (self.rss, self.sss):
            found = []
            try:
                for o in objs:
                    if (o.get("metadata") or {}).get("namespace", "") != ns:
                        continue
                    sel = label_selector_as_selector((o.get("spec") or {}).get("selector"))
                    if sel is NOTHING or sel == [] or not selector_matches(sel, lab):
                        continue      # nil / empty selectors match nothing here
                    found.append(sel)
            except AffinityError:
                found = []            # an invalid selector fails the whole lookup
            out.extend(found)
        return out


def selector_spread_map(pod, ni, selectors):
    """CalculateSpreadPriorityMap (selector_spreading.go:66-114): placed pods of the node in the
    pod's namespace, not being deleted, matching any of the selectors."""
    if not selectors:
        return 0
    ns = (pod.get("metadata") or {}).get("namespace", "")
    count = 0
    for q in ni.pods:
        md = q.get("metadata") or {}
        if md.get("namespace", "") != ns or md.get("deletionTimestamp") is not None:
            continue
        lab = md.get("labels") or {}
        if any(selector_matches(sel, lab) for sel in selectors):
            count += 1
    return count


def zone_key(node):
    """K/pkg/util/node GetZoneKey: region:\\x00:zone from failure-domain labels."""
    labels = (node.get("metadata") or {}).get("labels") or {}
    region = labels.get("failure-domain.beta.kubernetes.io/region", "")
    zone = labels.get("failure-domain.beta.kubernetes.io/zone", "")
    if region == "" and zone == "":
        return ""
    return region + ":\x00:" + zone


# Priority configs: name -> (kind, fn).  "map" = plain map; "reduce-rev"/"reduce-fwd"
# = NormalizeReduce; "spread" = selector spreading with no selectors in the
# simulator's store (map 0 → reduce); "const" = evaluates the same for every node
# under the simulator's inputs (documented in DESIGN.md).
def _prio_zero(pod, ni):
    return 0


PREFER_AVOID_KEY = "scheduler.alpha.kubernetes.io/preferAvoidPods"  # core/v1 annotation_key_constants.go


class _GoDecodeError(Exception):
    pass


def _go_obj(v):
    """encoding/json into a struct: a JSON object (kept as ordered pairs) or null."""
    if v is None or (isinstance(v, tuple) and v[0] == "obj"):
        return v
    raise _GoDecodeError("not an object")


def _go_get(o, name):
    """Field lookup of encoding/json: exact or case-insensitive key, later keys overwrite."""
    hit = None
    for k, v in o[1]:
        if k.lower() == name.lower():
            hit = (v,)
    return hit


def _go_str(o, name):
    h = _go_get(o, name)
    if h is None or h[0] is None:
        return ""
    if not isinstance(h[0], str):
        raise _GoDecodeError("not a string")
    return h[0]


def get_avoid_pods(annotations):
    """v1helper.GetAvoidPodsFromNodeAnnotations (pkg/apis/core/v1/helper/helpers.go:338-347):
    v1.AvoidPods from the node's annotation, or an error.  Entries are (kind, uid) of
    podSignature.podController, or None where that pointer stays nil (types.go AvoidPods /
    PreferAvoidPodsEntry / PodSignature)."""
    import json
    raw = (annotations or {}).get(PREFER_AVOID_KEY, "")
    if raw == "":
        return [], None
    try:
        doc = json.loads(raw, object_pairs_hook=lambda pairs: ("obj", pairs))
        top = _go_obj(doc)
        if top is None:
            return [], None
        h = _go_get(top, "preferAvoidPods")
        lst = None if h is None else h[0]
        if lst is None:
            return [], None
        if not isinstance(lst, list):
            raise _GoDecodeError("not an array")
        out = []
        for e in lst:
            e = _go_obj(e)
            ctl = None
            if e is not None:
                for f in ("reason", "message", "evictionTime"):
                    _go_str(e, f)
                hs = _go_get(e, "podSignature")
                sig = _go_obj(hs[0]) if hs is not None else None
                if sig is not None:
                    hc = _go_get(sig, "podController")
                    ctl = _go_obj(hc[0]) if hc is not None else None
            if ctl is None:
                out.append(None)
                continue
            for f in ("name", "apiVersion"):
                _go_str(ctl, f)
            for f in ("controller", "blockOwnerDeletion"):
                hb = _go_get(ctl, f)
                if hb is not None and hb[0] is not None and not isinstance(hb[0], bool):
                    raise _GoDecodeError("not a bool")
            out.append((_go_str(ctl, "kind"), _go_str(ctl, "uid")))
        return out, None
    except (ValueError, _GoDecodeError) as err:
        return [], err


def _prio_prefer_avoid(pod, ni):
    """CalculateNodePreferAvoidPodsPriorityMap (node_prefer_avoid_pods.go:32-68): the controllerRef
    (priorities/util/util.go:25-36, first ownerReference with controller=true) counts only for a
    ReplicationController / ReplicaSet; the node scores 0 when an annotation entry names the same
    (kind, uid), else MaxPriority (also when the annotation does not decode)."""
    ref = None
    for o in ((pod.get("metadata") or {}).get("ownerReferences") or []):
        if o.get("controller") is True:
            ref = o
            break
    if ref is None or ref.get("kind") not in ("ReplicationController", "ReplicaSet"):
        return MAX_PRIORITY
    avoids, err = get_avoid_pods((_meta(ni.node).get("annotations") or {}))
    if err is not None:
        return MAX_PRIORITY
    for sig in avoids:
        if sig is None:
            raise NotImplementedError("nil podController: the reference panics")
        if sig == (ref.get("kind"), ref.get("uid") or ""):
            return 0
    return MAX_PRIORITY


def _prio_equal(pod, ni):
    return 1


PRIORITIES = {
    "LeastRequestedPriority": ("map", prio_least_requested),
    "MostRequestedPriority": ("map", prio_most_requested),
    "BalancedResourceAllocation": ("map", prio_balanced),
    "TaintTolerationPriority": ("reduce-rev", prio_taint_toleration_map),
    "NodeAffinityPriority": ("reduce-fwd", prio_node_affinity_map),
    "NodePreferAvoidPodsPriority": ("map", _prio_prefer_avoid),
    "SelectorSpreadPriority": ("spread", _prio_zero),
    "ServiceSpreadingPriority": ("spread", _prio_zero),
    "InterPodAffinityPriority": ("ipa", None),
    "EqualPriority": ("map", _prio_equal),
    "ImageLocalityPriority": ("map", None),  # set below
}


MB = 1024 * 1024
MIN_IMG_SIZE, MAX_IMG_SIZE = 23 * MB, 1000 * MB   # image_locality.go:30-31


def prio_image_locality(pod, ni):
    """ImageLocalityPriorityMap (image_locality.go:39-88): the summed size of the pod's
    container images the node lists in status.images, bucketed 0..10."""
    sizes = {}
    for img in (ni.node.get("status") or {}).get("images") or []:
        for name in img.get("names") or []:
            sizes[name] = int(img.get("sizeBytes", 0))
    total = sum(sizes.get(c.get("image"), 0) for c in _containers(pod))
    if total == 0 or total < MIN_IMG_SIZE:
        return 0
    if total >= MAX_IMG_SIZE:
        return MAX_PRIORITY
    return (MAX_PRIORITY * (total - MIN_IMG_SIZE)) // (MAX_IMG_SIZE - MIN_IMG_SIZE) + 1


PRIORITIES["ImageLocalityPriority"] = ("map", prio_image_locality)


def node_label_priority(label, presence):
    """NodeLabelPrioritizer.CalculateNodeLabelPriorityMap (priorities/node_label.go:42-58): a Policy
    priority with a labelPreference argument."""
    def fn(pod, ni):
        exists = label in ((ni.node.get("metadata") or {}).get("labels") or {})
        return MAX_PRIORITY if exists == presence else 0
    return ("map", fn)


def service_anti_affinity_priority(label, spread=None):
    """ServiceAntiAffinity (selector_spreading.go:180-275, a Policy priority with a
    serviceAntiAffinity argument): per node the placed pods of the pod's first service
    (getFirstServiceSelector), reduced over the filtered nodes by the node's value of `label`."""
    def fn(pod, infos):
        sel = None
        if spread is not None:
            md = pod.get("metadata") or {}
            ns, lab = md.get("namespace", ""), md.get("labels") or {}
            for svc in spread.services:
                s = (svc.get("spec") or {}).get("selector")
                if (svc.get("metadata") or {}).get("namespace", "") == ns and s is not None and \
                        SpreadListers._set_matches(s, lab):
                    sel = selector_from_set(s)
                    break
        ns = (pod.get("metadata") or {}).get("namespace", "")
        counts = []
        for ni in infos:
            c = 0
            if sel is not None:
                for q in ni.pods:
                    qm = q.get("metadata") or {}
                    if qm.get("namespace", "") == ns and selector_matches(sel, qm.get("labels") or {}):
                        c += 1
            counts.append(c)
        total = sum(counts)
        per_label = {}
        vals = []
        for ni, c in zip(infos, counts):
            lab = (ni.node.get("metadata") or {}).get("labels") or {}
            v = lab.get(label) if label in lab else None
            vals.append(v)
            if v is not None:
                per_label[v] = per_label.get(v, 0) + c
        out = []
        for v in vals:
            if v is None:
                out.append(0)
                continue
            f = float(MAX_PRIORITY)
            if total > 0:
                f = float(MAX_PRIORITY) * (float(total - per_label[v]) / float(total))
            out.append(int(f))
        return out
    return ("function", fn)


def prioritize_nodes(pod, infos, configs, all_infos=None, hard_weight=10, spread=None, custom=None):
    """S/core/generic_scheduler.go:542-676.  configs: list of (name, weight); infos: the
    filtered nodes; all_infos: nodeNameToInfo (InterPodAffinityPriority reads every pod);
    spread: SpreadListers for SelectorSpread / ServiceSpreading (None: the simulator's empty ones);
    custom: Policy priorities registered with an argument, by name (node_label_priority, ...)."""
    if not configs:
        return [1 for _ in infos]          # EqualPriorityMap
    total = [0] * len(infos)
    for name, weight in configs:
        kind, fn = custom[name] if custom and name in custom else PRIORITIES[name]
        if kind == "function":
            scores = fn(pod, infos)
        elif kind == "ipa":
            scores = interpod_affinity_priority(pod, all_infos if all_infos is not None else infos,
                                                [ni.node for ni in infos], hard_weight)
        elif kind == "spread":
            # ServiceSpreadingPriority: services only (factory/plugins.go registers it with empty
            # controller listers, defaults.go:68-74)
            sels = spread.selectors(pod, name == "ServiceSpreadingPriority") if spread is not None else []
            scores = [selector_spread_map(pod, ni, sels) for ni in infos]
        else:
            scores = [fn(pod, ni) for ni in infos]
        if kind == "reduce-rev":
            scores = normalize_reduce(scores, True)
        elif kind == "reduce-fwd":
            scores = normalize_reduce(scores, False)
        elif kind == "spread":
            scores = spread_reduce(scores, [zone_key(ni.node) for ni in infos])
        for i, s in enumerate(scores):
            total[i] += s * weight
    return total


# --------------------------------------------------------------------------
# Providers (S/algorithmprovider/defaults/defaults.go:113-259)
# --------------------------------------------------------------------------
DEFAULT_PREDICATES = {"NoVolumeZoneConflict", "MaxEBSVolumeCount", "MaxGCEPDVolumeCount",
                      "MaxAzureDiskVolumeCount", "MatchInterPodAffinity", "NoDiskConflict",
                      "GeneralPredicates", "CheckNodeMemoryPressure", "CheckNodeDiskPressure",
                      "CheckNodeCondition", "PodToleratesNodeTaints", "CheckVolumeBinding"}
DEFAULT_PRIORITIES = [("SelectorSpreadPriority", 1), ("InterPodAffinityPriority", 1),
                      ("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1),
                      ("NodePreferAvoidPodsPriority", 10000), ("NodeAffinityPriority", 1),
                      ("TaintTolerationPriority", 1)]


def provider(name):
    pri = list(DEFAULT_PRIORITIES)
    if name in ("ClusterAutoscalerProvider", "TalkintDataProvider"):
        pri = [("MostRequestedPriority", 1) if n == "LeastRequestedPriority" else (n, w) for n, w in pri]
    elif name != "DefaultProvider":
        raise KeyError(name)
    return set(DEFAULT_PREDICATES), pri


# --------------------------------------------------------------------------
# Generic scheduler (S/core/generic_scheduler.go:112-198)
# --------------------------------------------------------------------------
class FitError(Exception):
    def __init__(self, num_nodes, failed):
        self.num_nodes = num_nodes
        self.failed = failed      # node name -> [reasons]

    def histogram(self):
        h = {}
        for rs in self.failed.values():
            for r in rs:
                h[r] = h.get(r, 0) + 1
        return h

    def __str__(self):
        """FitError.Error (generic_scheduler.go:72-90)."""
        parts = sorted("%d %s" % (v, k) for k, v in self.histogram().items())
        return "0/%d nodes are available: %s." % (self.num_nodes, ", ".join(parts))


class GenericScheduler:
    def __init__(self, predicate_keys, priority_configs, custom_predicates=None, hard_weight=10, spread=None,
                 custom_priorities=None):
        self.predicates = set(predicate_keys) | set(MANDATORY_PREDICATES)
        self.spread = spread              # SpreadListers (None: the simulator's empty listers)
        self.custom_priorities = custom_priorities
        self.custom = dict(custom_predicates or {})
        self.prioritizers = list(priority_configs)
        self.hard_weight = hard_weight    # hardPodAffinitySymmetricWeight (simulator: 10)
        self.last_node_index = 0          # uint64 (generic_scheduler.go:102)

    def schedule(self, pod, infos):
        """Schedule (generic_scheduler.go:112-167). infos: list of NodeInfo in any order (the
        listed nodes; every cached pod sits on one of them)."""
        if not infos:
            raise RuntimeError("no nodes available to schedule pods")
        custom = self.custom
        if "MatchInterPodAffinity" in self.predicates and "MatchInterPodAffinity" not in custom:
            # the predicate metadata (GetMetadata, metadata.go:102-123: existing pods' anti-affinity
            # terms, from PodsWithAffinity) once per pod, then the checker per node with the
            # cache's pods as the pod lister; trivially true without terms on either side
            meta = matching_anti_affinity_terms(pod, [(p, ni.node) for ni in infos for p in ni.pods_with_affinity])
            if meta or has_pod_affinity_constraints(pod):
                all_pods = [(p, ni.node) for ni in infos for p in ni.pods]
                custom = dict(custom, MatchInterPodAffinity=_interpod_predicate(meta, all_pods))
        filtered, failed = [], {}
        for ni in infos:
            ok, rs = pod_fits_on_node(pod, ni, self.predicates, custom) if self.predicates else (True, [])
            if ok:
                filtered.append(ni)
            else:
                failed[ni.name] = rs
        if not filtered:
            raise FitError(len(infos), failed)
        if len(filtered) == 1:
            return filtered[0].name
        scores = prioritize_nodes(pod, filtered, self.prioritizers, infos, self.hard_weight, self.spread,
                                  self.custom_priorities)
        return self.select_host([(ni.name, s) for ni, s in zip(filtered, scores)])

    def select_host(self, plist):
        """selectHost (generic_scheduler.go:183-198) + HostPriorityList.Less (S/api/types.go:272-277).
        Host names compare bytewise (Go string <)."""
        lst = sorted(plist, key=lambda hs: (hs[1], hs[0].encode()), reverse=True)
        mx = lst[0][1]
        first_after = next((i for i, hs in enumerate(lst) if hs[1] < mx), len(lst))
        ix = self.last_node_index % first_after
        self.last_node_index = (self.last_node_index + 1) % (1 << 64)
        return lst[ix][0]


# --------------------------------------------------------------------------
# Scheduler cache (S/schedulercache/cache.go) driven by informer-style events, and the
# scheduleOne loop's Schedule + assume (S/scheduler.go:188-204, 366-397)
# --------------------------------------------------------------------------
class SchedulerCache:
    def __init__(self, predicate_keys, priority_configs, custom_predicates=None, spread=None):
        self.nodes = {}          # name -> NodeInfo (cache.nodes)
        self.listed = []         # names the node lister returns (added, not removed)
        self.pod_states = {}     # key -> pod
        self.assumed = set()
        self.sched = GenericScheduler(predicate_keys, priority_configs, custom_predicates, spread=spread)

    def _info(self, name):
        n = self.nodes.get(name)
        if n is None:
            n = self.nodes[name] = NodeInfo()
        return n

    def _add(self, pod):                                   # cache.go:200-207
        self._info((pod.get("spec") or {}).get("nodeName", "")).add_pod(pod)

    def _remove(self, pod):                                # cache.go:219-228
        name = (pod.get("spec") or {}).get("nodeName", "")
        n = self.nodes[name]
        n.remove_pod(pod)
        if not n.pods and n.node is None:
            del self.nodes[name]

    def assume_pod(self, pod):                             # cache.go:125-143
        key = pod_key(pod)
        if key in self.pod_states:
            raise KeyError("pod %s is in the cache, so can't be assumed" % key)
        self._add(pod)
        self.pod_states[key] = pod
        self.assumed.add(key)

    def add_pod(self, pod):                                # cache.go:230-262
        key = pod_key(pod)
        cur = self.pod_states.get(key)
        if cur is not None and key in self.assumed:
            if (cur.get("spec") or {}).get("nodeName") != (pod.get("spec") or {}).get("nodeName"):
                self._remove(cur)
                self._add(pod)
            self.assumed.discard(key)
            self.pod_states[key] = pod
        elif cur is None:
            self._add(pod)
            self.pod_states[key] = pod
        else:
            raise KeyError("pod %s was already in added state" % key)

    def update_pod(self, old, new):                        # cache.go:265-289
        key = pod_key(old)
        if key not in self.pod_states or key in self.assumed:
            raise KeyError("pod %s is not added to scheduler cache, so cannot be updated" % key)
        self._remove(old)
        self._add(new)
        self.pod_states[key] = new

    def remove_pod(self, pod):                             # cache.go:292-318
        key = pod_key(pod)
        cur = self.pod_states.get(key)
        if cur is None or key in self.assumed:
            raise KeyError("pod %s is not found in scheduler cache, so cannot be removed from it" % key)
        self._remove(cur)
        del self.pod_states[key]

    def forget_pod(self, pod):                             # cache.go:170-197 (scheduler.go:412: the bind failed)
        key = pod_key(pod)
        cur = self.pod_states.get(key)
        if cur is not None and (cur.get("spec") or {}).get("nodeName") != (pod.get("spec") or {}).get("nodeName"):
            raise KeyError("pod %s was assumed on %s but assigned to %s" % (key, (pod.get("spec") or {}).get("nodeName"),
                                                                          (cur.get("spec") or {}).get("nodeName")))
        if cur is None or key not in self.assumed:
            raise KeyError("pod %s wasn't assumed so cannot be forgotten" % key)
        self._remove(pod)
        self.assumed.discard(key)
        del self.pod_states[key]

    def add_node(self, node):                              # cache.go:354-363
        name = (node.get("metadata") or {}).get("name", "")
        self._info(name).set_node(node)
        if name not in self.listed:
            self.listed.append(name)

    def update_node(self, old, new):                       # cache.go:366-375
        self.add_node(new)

    def remove_node(self, node):                           # cache.go:378-393
        name = (node.get("metadata") or {}).get("name", "")
        n = self.nodes[name]
        n.remove_node()
        if not n.pods and n.node is None:
            del self.nodes[name]
        self.listed.remove(name)

    def schedule(self, pod):
        """genericScheduler.Schedule over the listed nodes (nodeLister.List, factory.go:1088)."""
        return self.sched.schedule(pod, [self.nodes[n] for n in self.listed])

    def schedule_one(self, pod):
        """scheduleOne's schedule + assume (scheduler.go:431-484): returns the host, or the
        FitError message; the assumed pod carries spec.nodeName = host."""
        try:
            host = self.schedule(pod)
        except FitError as e:
            return None, str(e)
        assumed = dict(pod)
        assumed["spec"] = dict(pod.get("spec") or {}, nodeName=host)
        self.assume_pod(assumed)
        return host, None


# --------------------------------------------------------------------------
# Simulator (pkg/scheduler/simulator.go:108-223, pkg/framework/store/store.go:212-241)
# --------------------------------------------------------------------------
def expand_simulation_pods(spec_list):
    """cmd/app/options/options.go:73-99: each SimulationPod repeated Num times,
    labelled SimulationName=<name>, namespace "" (names are uuids in Go; here
    deterministic <name>-<i>)."""
    out = []
    for sp in spec_list:
        for i in range(int(sp.get("num", 0))):
            pod = {"metadata": {"name": "%s-%d" % (sp["name"], i), "namespace": "",
                                "labels": {"SimulationName": sp["name"]}},
                   "spec": (sp.get("pod") or {}).get("spec") or {}}
            out.append(pod)
    return out


def simulate(nodes, running_pods, sim_pods, predicate_keys, priority_configs, custom_predicates=None, spread=None,
             custom_priorities=None):
    """Runs the ClusterCapacity loop: pods are popped LIFO (store.go:223-233),
    each is scheduled, bound pods are assumed into the node cache (scheduler.go:366
    → cache.go:125 → node_info.go:318), unschedulable pods are recorded and the
    loop continues (simulator.go:163-185) until the queue is empty.
    Returns list of (pod_name, node_name or None, fit_error_message or None)."""
    infos = [NodeInfo(n) for n in nodes]
    by_name = {ni.name: ni for ni in infos}
    for p in running_pods:
        nn = (p.get("spec") or {}).get("nodeName", "")
        if nn in by_name:
            by_name[nn].add_pod(p)
    sched = GenericScheduler(predicate_keys, priority_configs, custom_predicates, spread=spread,
                             custom_priorities=custom_priorities)
    queue = list(sim_pods)
    out = []
    while queue:
        pod = queue.pop()
        name = (pod.get("metadata") or {}).get("name", "")
        try:
            host = sched.schedule(pod, infos)
        except FitError as e:
            out.append((name, None, str(e)))
            continue
        by_name[host].add_pod(pod)
        out.append((name, host, None))
    return out, sched.last_node_index
