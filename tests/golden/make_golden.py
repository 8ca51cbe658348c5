"""Generates tests/golden/*.json — golden vectors hand-transcribed from the reference's
own Go unit tests (the vendored kube-scheduler v1.10 tests under
/root/reference/vendor/k8s.io/kubernetes/pkg/scheduler/).  Each case records the Go
test function and file:line it was transcribed from.  Inputs are rebuilt here as
Kubernetes-shaped JSON objects with the helpers the Go tests use (makeNode,
newResourcePod, newPod, ...); expected outputs are copied verbatim.

Run:  python tests/golden/make_golden.py      (rewrites the JSON files)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

HERE = os.path.dirname(os.path.abspath(__file__))
S = "vendor/k8s.io/kubernetes/pkg/scheduler/"


# ---------------------------------------------------------------- helpers
def node(name="", cpu_m=None, mem=None, pods=None, labels=None, taints=None, conditions=None,
         unschedulable=None, alloc_extra=None):
    n = {"metadata": {"name": name}, "spec": {}, "status": {}}
    alloc = {}
    if cpu_m is not None:
        alloc["cpu"] = "%dm" % cpu_m
    if mem is not None:
        alloc["memory"] = "%d" % mem
    if pods is not None:
        alloc["pods"] = "%d" % pods
    if alloc_extra:
        alloc.update(alloc_extra)
    if alloc:
        n["status"]["allocatable"] = alloc
    if labels is not None:
        n["metadata"]["labels"] = labels
    if taints is not None:
        n["spec"]["taints"] = taints
    if conditions is not None:
        n["status"]["conditions"] = [{"type": t, "status": s} for t, s in conditions]
    if unschedulable is not None:
        n["spec"]["unschedulable"] = unschedulable
    return n


def ctr(cpu=None, mem=None, extra=None, ports=None):
    """A container whose requests hold exactly the given quantity strings."""
    req = {}
    if cpu is not None:
        req["cpu"] = cpu
    if mem is not None:
        req["memory"] = mem
    if extra:
        req.update(extra)
    c = {"resources": {"requests": req}} if (req or cpu is not None or mem is not None) else {}
    if ports:
        c["ports"] = ports
    return c


def pod(containers=None, init=None, node_name=None, name=None, labels=None, **spec):
    p = {"metadata": {}, "spec": {}}
    if name:
        p["metadata"]["name"] = name
    if labels:
        p["metadata"]["labels"] = labels
    if containers is not None:
        p["spec"]["containers"] = containers
    if init is not None:
        p["spec"]["initContainers"] = init
    if node_name:
        p["spec"]["nodeName"] = node_name
    p["spec"].update(spec)
    return p


def res_ctr(cpu_m=0, mem=0, scalar=None, eph=None):
    """Container built from schedulercache.Resource.ResourceList() (node_info.go:111-127):
    cpu, memory, nvidia-gpu, pods and ephemeral-storage are ALWAYS present (zero or not)."""
    req = {"cpu": "%dm" % cpu_m, "memory": "%d" % mem, "alpha.kubernetes.io/nvidia-gpu": "0",
           "pods": "0", "ephemeral-storage": "%d" % (eph or 0)}
    for k, v in (scalar or {}).items():
        req[k] = "%d" % v
    return {"resources": {"requests": req}}


cases = {}


def add(group, case):
    cases.setdefault(group, []).append(case)


# ------------------------------------------------ priorities: LR / MR / BRA
# least_requested_test.go:30-245, most_requested_test.go:30-206,
# balanced_resource_allocation_test.go:30-264 share these pod specs.
no_resources = pod(containers=[])
cpu_only = pod(node_name="machine1", containers=[ctr("1000m", "0"), ctr("2000m", "0")])
cpu_only2 = pod(node_name="machine2", containers=[ctr("1000m", "0"), ctr("2000m", "0")])
cpu_and_memory = pod(node_name="machine2", containers=[ctr("1000m", "2000"), ctr("2000m", "3000")])
big_cpu_and_memory = pod(node_name="machine1", containers=[ctr("2000m", "4000"), ctr("3000m", "5000")])
m1 = pod(node_name="machine1")
m2 = pod(node_name="machine2")


def mk(name, c, m):   # priorities/test_util.go:28 makeNode (no pods entry)
    return node(name, c, m)


def prio_case(src, prio, test, p, nodes, expect, pods=()):
    add("priorities", {"source": src, "test": test, "priority": prio, "pod": p,
                       "nodes": nodes, "pods": list(pods), "expect": expect})


LRsrc = S + "algorithm/priorities/least_requested_test.go"
prio_case(LRsrc + ":111", "LeastRequestedPriority", "nothing scheduled, nothing requested", no_resources,
          [mk("machine1", 4000, 10000), mk("machine2", 4000, 10000)], [["machine1", 10], ["machine2", 10]])
prio_case(LRsrc + ":125", "LeastRequestedPriority", "nothing scheduled, resources requested, differently sized machines",
          cpu_and_memory, [mk("machine1", 4000, 10000), mk("machine2", 6000, 10000)], [["machine1", 3], ["machine2", 5]])
prio_case(LRsrc + ":139", "LeastRequestedPriority", "no resources requested, pods scheduled", no_resources,
          [mk("machine1", 4000, 10000), mk("machine2", 4000, 10000)], [["machine1", 10], ["machine2", 10]],
          [m1, m1, m2, m2])
prio_case(LRsrc + ":159", "LeastRequestedPriority", "no resources requested, pods scheduled with resources", no_resources,
          [mk("machine1", 10000, 20000), mk("machine2", 10000, 20000)], [["machine1", 7], ["machine2", 5]],
          [cpu_only, cpu_only, cpu_only2, cpu_and_memory])
prio_case(LRsrc + ":179", "LeastRequestedPriority", "resources requested, pods scheduled with resources", cpu_and_memory,
          [mk("machine1", 10000, 20000), mk("machine2", 10000, 20000)], [["machine1", 5], ["machine2", 4]],
          [cpu_only, cpu_and_memory])
prio_case(LRsrc + ":197", "LeastRequestedPriority", "resources requested, pods scheduled with resources, differently sized machines",
          cpu_and_memory, [mk("machine1", 10000, 20000), mk("machine2", 10000, 50000)], [["machine1", 5], ["machine2", 6]],
          [cpu_only, cpu_and_memory])
prio_case(LRsrc + ":215", "LeastRequestedPriority", "requested resources exceed node capacity", cpu_only,
          [mk("machine1", 4000, 10000), mk("machine2", 4000, 10000)], [["machine1", 5], ["machine2", 2]],
          [cpu_only, cpu_and_memory])
prio_case(LRsrc + ":224", "LeastRequestedPriority", "zero node resources, pods scheduled with resources", no_resources,
          [mk("machine1", 0, 0), mk("machine2", 0, 0)], [["machine1", 0], ["machine2", 0]],
          [cpu_only, cpu_and_memory])

MRsrc = S + "algorithm/priorities/most_requested_test.go"
prio_case(MRsrc + ":128", "MostRequestedPriority", "nothing scheduled, nothing requested", no_resources,
          [mk("machine1", 4000, 10000), mk("machine2", 4000, 10000)], [["machine1", 0], ["machine2", 0]])
prio_case(MRsrc + ":142", "MostRequestedPriority", "nothing scheduled, resources requested, differently sized machines",
          cpu_and_memory, [mk("machine1", 4000, 10000), mk("machine2", 6000, 10000)], [["machine1", 6], ["machine2", 5]])
prio_case(MRsrc + ":156", "MostRequestedPriority", "no resources requested, pods scheduled with resources", no_resources,
          [mk("machine1", 10000, 20000), mk("machine2", 10000, 20000)], [["machine1", 3], ["machine2", 4]],
          [cpu_only, cpu_only, cpu_only2, cpu_and_memory])
prio_case(MRsrc + ":176", "MostRequestedPriority", "resources requested, pods scheduled with resources", cpu_and_memory,
          [mk("machine1", 10000, 20000), mk("machine2", 10000, 20000)], [["machine1", 4], ["machine2", 5]],
          [cpu_only, cpu_and_memory])
prio_case(MRsrc + ":194", "MostRequestedPriority", "resources requested with more than the node, pods scheduled with resources",
          big_cpu_and_memory, [mk("machine1", 4000, 10000), mk("machine2", 10000, 8000)], [["machine1", 4], ["machine2", 2]])

BRsrc = S + "algorithm/priorities/balanced_resource_allocation_test.go"
prio_case(BRsrc + ":116", "BalancedResourceAllocation", "nothing scheduled, nothing requested", no_resources,
          [mk("machine1", 4000, 10000), mk("machine2", 4000, 10000)], [["machine1", 10], ["machine2", 10]])
prio_case(BRsrc + ":133", "BalancedResourceAllocation", "nothing scheduled, resources requested, differently sized machines",
          cpu_and_memory, [mk("machine1", 4000, 10000), mk("machine2", 6000, 10000)], [["machine1", 7], ["machine2", 10]])
prio_case(BRsrc + ":150", "BalancedResourceAllocation", "no resources requested, pods scheduled", no_resources,
          [mk("machine1", 4000, 10000), mk("machine2", 4000, 10000)], [["machine1", 10], ["machine2", 10]],
          [m1, m1, m2, m2])
prio_case(BRsrc + ":173", "BalancedResourceAllocation", "no resources requested, pods scheduled with resources", no_resources,
          [mk("machine1", 10000, 20000), mk("machine2", 10000, 20000)], [["machine1", 4], ["machine2", 6]],
          [cpu_only, cpu_only, cpu_only2, cpu_and_memory])
prio_case(BRsrc + ":196", "BalancedResourceAllocation", "resources requested, pods scheduled with resources", cpu_and_memory,
          [mk("machine1", 10000, 20000), mk("machine2", 10000, 20000)], [["machine1", 6], ["machine2", 9]],
          [cpu_only, cpu_and_memory])
prio_case(BRsrc + ":217", "BalancedResourceAllocation", "resources requested, pods scheduled with resources, differently sized machines",
          cpu_and_memory, [mk("machine1", 10000, 20000), mk("machine2", 10000, 50000)], [["machine1", 6], ["machine2", 6]],
          [cpu_only, cpu_and_memory])
prio_case(BRsrc + ":238", "BalancedResourceAllocation", "requested resources exceed node capacity", cpu_only,
          [mk("machine1", 4000, 10000), mk("machine2", 4000, 10000)], [["machine1", 0], ["machine2", 0]],
          [cpu_only, cpu_and_memory])
prio_case(BRsrc + ":247", "BalancedResourceAllocation", "zero node resources, pods scheduled with resources", no_resources,
          [mk("machine1", 0, 0), mk("machine2", 0, 0)], [["machine1", 0], ["machine2", 0]],
          [cpu_only, cpu_and_memory])

# ------------------------------------------------ TaintToleration priority
TTsrc = S + "algorithm/priorities/taint_toleration_test.go"


def tnode(name, taints):
    return node(name, taints=taints)


def taint(k, v, e):
    return {"key": k, "value": v, "effect": e}


def tol(k, op, v, e):
    d = {"key": k, "operator": op, "value": v}
    if e:
        d["effect"] = e
    return d


prio_case(TTsrc + ":51", "TaintTolerationPriority",
          "node with taints tolerated by the pod, gets a higher score than those node with intolerable taints",
          pod(tolerations=[tol("foo", "Equal", "bar", "PreferNoSchedule")]),
          [tnode("nodeA", [taint("foo", "bar", "PreferNoSchedule")]), tnode("nodeB", [taint("foo", "blah", "PreferNoSchedule")])],
          [["nodeA", 10], ["nodeB", 0]])
prio_case(TTsrc + ":75", "TaintTolerationPriority",
          "the nodes that all of their taints are tolerated by the pod, get the same score, no matter how many tolerable taints a node has",
          pod(tolerations=[tol("cpu-type", "Equal", "arm64", "PreferNoSchedule"), tol("disk-type", "Equal", "ssd", "PreferNoSchedule")]),
          [tnode("nodeA", []), tnode("nodeB", [taint("cpu-type", "arm64", "PreferNoSchedule")]),
           tnode("nodeC", [taint("cpu-type", "arm64", "PreferNoSchedule"), taint("disk-type", "ssd", "PreferNoSchedule")])],
          [["nodeA", 10], ["nodeB", 10], ["nodeC", 10]])
prio_case(TTsrc + ":118", "TaintTolerationPriority", "the more intolerable taints a node has, the lower score it gets.",
          pod(tolerations=[tol("foo", "Equal", "bar", "PreferNoSchedule")]),
          [tnode("nodeA", []), tnode("nodeB", [taint("cpu-type", "arm64", "PreferNoSchedule")]),
           tnode("nodeC", [taint("cpu-type", "arm64", "PreferNoSchedule"), taint("disk-type", "ssd", "PreferNoSchedule")])],
          [["nodeA", 10], ["nodeB", 5], ["nodeC", 0]])
prio_case(TTsrc + ":154", "TaintTolerationPriority",
          "only taints and tolerations that have effect PreferNoSchedule are checked by taints-tolerations priority function",
          pod(tolerations=[tol("cpu-type", "Equal", "arm64", "NoSchedule"), tol("disk-type", "Equal", "ssd", "NoSchedule")]),
          [tnode("nodeA", []), tnode("nodeB", [taint("cpu-type", "arm64", "NoSchedule")]),
           tnode("nodeC", [taint("cpu-type", "arm64", "PreferNoSchedule"), taint("disk-type", "ssd", "PreferNoSchedule")])],
          [["nodeA", 10], ["nodeB", 10], ["nodeC", 0]])
prio_case(TTsrc + ":196", "TaintTolerationPriority", "Default behaviour No taints and tolerations, lands on node with no taints",
          pod(tolerations=[]),
          [tnode("nodeA", []), tnode("nodeB", [taint("cpu-type", "arm64", "PreferNoSchedule")])],
          [["nodeA", 10], ["nodeB", 0]])

# ------------------------------------------------ NodeAffinity priority
NAsrc = S + "algorithm/priorities/node_affinity_test.go"


def pref(w, exprs):
    return {"weight": w, "preference": {"matchExpressions": exprs}}


def expr(k, op, vals=None):
    e = {"key": k, "operator": op}
    if vals is not None:
        e["values"] = vals
    return e


aff1 = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [pref(2, [expr("foo", "In", ["bar"])])]}}
aff2 = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
    pref(2, [expr("foo", "In", ["bar"])]), pref(4, [expr("key", "In", ["value"])]),
    pref(5, [expr("foo", "In", ["bar"]), expr("key", "In", ["value"]), expr("az", "In", ["az1"])])]}}
L1, L2, L3 = {"foo": "bar"}, {"key": "value"}, {"az": "az1"}
L4 = {"abc": "az11", "def": "az22"}
L5 = {"foo": "bar", "key": "value", "az": "az1"}
prio_case(NAsrc + ":127", "NodeAffinityPriority", "all machines are same priority as NodeAffinity is nil", pod(),
          [node("machine1", labels=L1), node("machine2", labels=L2), node("machine3", labels=L3)],
          [["machine1", 0], ["machine2", 0], ["machine3", 0]])
prio_case(NAsrc + ":141", "NodeAffinityPriority",
          "no machine macthes preferred scheduling requirements in NodeAffinity of pod so all machines' priority is zero",
          pod(affinity=aff1), [node("machine1", labels=L4), node("machine2", labels=L2), node("machine3", labels=L3)],
          [["machine1", 0], ["machine2", 0], ["machine3", 0]])
prio_case(NAsrc + ":155", "NodeAffinityPriority", "only machine1 matches the preferred scheduling requirements of pod",
          pod(affinity=aff1), [node("machine1", labels=L1), node("machine2", labels=L2), node("machine3", labels=L3)],
          [["machine1", 10], ["machine2", 0], ["machine3", 0]])
prio_case(NAsrc + ":169", "NodeAffinityPriority",
          "all machines matches the preferred scheduling requirements of pod but with different priorities ",
          pod(affinity=aff2), [node("machine1", labels=L1), node("machine5", labels=L5), node("machine2", labels=L2)],
          [["machine1", 1], ["machine5", 10], ["machine2", 3]])

# ------------------------------------------------ NodePreferAvoidPods
PAsrc = S + "algorithm/priorities/node_prefer_avoid_pods_test.go"
PA_KEY = "scheduler.alpha.kubernetes.io/preferAvoidPods"   # v1.PreferAvoidPodsAnnotationKey


def pa_annotation(kind, uid):   # node_prefer_avoid_pods_test.go:31-70 (whitespace dropped)
    return {PA_KEY: json.dumps({"preferAvoidPods": [{
        "podSignature": {"podController": {"apiVersion": "v1", "kind": kind, "name": "foo", "uid": uid,
                                           "controller": True}},
        "reason": "some reason", "message": "some message"}]})}


def pa_node(name, ann=None):
    n = node(name)
    if ann:
        n["metadata"]["annotations"] = ann
    return n


def owned(kind, uid, controller=True):
    p = pod()
    ref = {"kind": kind, "name": "foo", "uid": uid}
    if controller:
        ref["controller"] = True
    p["metadata"]["namespace"] = "default"
    p["metadata"]["ownerReferences"] = [ref]
    return p


PA_NODES = [pa_node("machine1", pa_annotation("ReplicationController", "abcdef123456")),
            pa_node("machine2", pa_annotation("ReplicaSet", "qwert12345")), pa_node("machine3")]
prio_case(PAsrc + ":89", "NodePreferAvoidPodsPriority",
          "pod managed by ReplicationController should avoid a node, this node get lowest priority score",
          owned("ReplicationController", "abcdef123456"), PA_NODES, [["machine1", 0], ["machine2", 10], ["machine3", 10]])
prio_case(PAsrc + ":102", "NodePreferAvoidPodsPriority", "ownership by random controller should be ignored",
          owned("RandomController", "abcdef123456"), PA_NODES, [["machine1", 10], ["machine2", 10], ["machine3", 10]])
prio_case(PAsrc + ":115", "NodePreferAvoidPodsPriority", "owner without Controller field set should be ignored",
          owned("ReplicationController", "abcdef123456", controller=False), PA_NODES,
          [["machine1", 10], ["machine2", 10], ["machine3", 10]])
prio_case(PAsrc + ":128", "NodePreferAvoidPodsPriority",
          "pod managed by ReplicaSet should avoid a node, this node get lowest priority score",
          owned("ReplicaSet", "qwert12345"), PA_NODES, [["machine1", 10], ["machine2", 0], ["machine3", 10]])


# ------------------------------------------------ ImageLocality
ILsrc = S + "algorithm/priorities/image_locality_test.go"
MiB = 1024 * 1024


def img_node(name, images):   # makeImageNode (image_locality_test.go:203-208)
    n = node(name)
    n["status"]["images"] = [{"names": names, "sizeBytes": size} for names, size in images]
    return n


def img_pod(*images):
    return pod(containers=[{"image": i} for i in images])


IL_N1 = [(["gcr.io/40", "gcr.io/40:v1", "gcr.io/40:v1"], 40 * MiB), (["gcr.io/140", "gcr.io/140:v1"], 140 * MiB),
         (["gcr.io/2000"], 2000 * MiB)]                                   # node401402000 (:68-92)
IL_N2 = [(["gcr.io/250"], 250 * MiB), (["gcr.io/10", "gcr.io/10:v1"], 10 * MiB)]   # node25010 (:94-109)
IL_NODES = [img_node("machine1", IL_N1), img_node("machine2", IL_N2)]
prio_case(ILsrc + ":130", "ImageLocalityPriority", "two images spread on two nodes, prefer the larger image one",
          img_pod("gcr.io/40", "gcr.io/250"), IL_NODES, [["machine1", 1], ["machine2", 3]])
prio_case(ILsrc + ":145", "ImageLocalityPriority", "two images on one node, prefer this node",
          img_pod("gcr.io/40", "gcr.io/140"), IL_NODES, [["machine1", 2], ["machine2", 0]])
prio_case(ILsrc + ":160", "ImageLocalityPriority", "if exceed limit, use limit",
          img_pod("gcr.io/10", "gcr.io/2000"), IL_NODES, [["machine1", 10], ["machine2", 0]])

# ------------------------------------------------ PodFitsResources
PFsrc = S + "algorithm/predicates/predicates_test.go"
EXT_A, EXT_B, HUGE_A = "example.com/aaa", "example.com/bbb", "hugepages-2Mi"


def alloc(cpu, mem, gpu, pods, ext_a, eph, huge_a):   # predicates_test.go:62-72
    return {"cpu": "%dm" % cpu, "memory": "%d" % mem, "pods": "%d" % pods,
            "alpha.kubernetes.io/nvidia-gpu": "%d" % gpu, EXT_A: "%d" % ext_a,
            "ephemeral-storage": "%d" % eph, HUGE_A: "%d" % huge_a}


def rpod(*usages, init=None):
    p = pod(containers=[res_ctr(**u) for u in usages])
    if init is not None:
        p["spec"]["initContainers"] = [res_ctr(**u) for u in init]
    return p


def R(c=0, m=0, **kw):
    d = {"cpu_m": c, "mem": m}
    d.update(kw)
    return d


def fit_case(src, test, p, existing, nalloc, fits, reasons=()):
    n = {"metadata": {"name": "n"}, "spec": {}, "status": {"allocatable": nalloc}}
    ex = []
    for e in existing:
        e = json.loads(json.dumps(e))
        e["spec"]["nodeName"] = "n"
        ex.append(e)
    add("predicates", {"source": src, "test": test, "predicate": "PodFitsResources", "pod": p,
                       "node": n, "pods": ex, "fits": fits, "reasons": list(reasons)})


A32 = alloc(10, 20, 0, 32, 5, 20, 5)
IC, IM, IP, IE = "Insufficient cpu", "Insufficient memory", "Insufficient pods", "Insufficient ephemeral-storage"
fit_case(PFsrc + ":104", "no resources requested always fits", pod(), [rpod(R(10, 20))], A32, True)
fit_case(PFsrc + ":111", "too many resources fails", rpod(R(1, 1)), [rpod(R(10, 20))], A32, False, [IC, IM])
fit_case(PFsrc + ":121", "too many resources fails due to init container cpu", rpod(R(1, 1), init=[R(3, 1)]),
         [rpod(R(8, 19))], A32, False, [IC])
fit_case(PFsrc + ":128", "too many resources fails due to highest init container cpu",
         rpod(R(1, 1), init=[R(3, 1), R(2, 1)]), [rpod(R(8, 19))], A32, False, [IC])
fit_case(PFsrc + ":135", "too many resources fails due to init container memory", rpod(R(1, 1), init=[R(1, 3)]),
         [rpod(R(9, 19))], A32, False, [IM])
fit_case(PFsrc + ":142", "too many resources fails due to highest init container memory",
         rpod(R(1, 1), init=[R(1, 3), R(1, 2)]), [rpod(R(9, 19))], A32, False, [IM])
fit_case(PFsrc + ":149", "init container fits because it's the max, not sum, of containers and init containers",
         rpod(R(1, 1), init=[R(1, 1)]), [rpod(R(9, 19))], A32, True)
fit_case(PFsrc + ":155", "multiple init containers fit because it's the max, not sum, of containers and init containers",
         rpod(R(1, 1), init=[R(1, 1), R(1, 1)]), [rpod(R(9, 19))], A32, True)
fit_case(PFsrc + ":161", "both resources fit", rpod(R(1, 1)), [rpod(R(5, 5))], A32, True)
fit_case(PFsrc + ":167", "one resource memory fits", rpod(R(2, 1)), [rpod(R(9, 5))], A32, False, [IC])
fit_case(PFsrc + ":174", "one resource cpu fits", rpod(R(1, 2)), [rpod(R(5, 19))], A32, False, [IM])
fit_case(PFsrc + ":181", "equal edge case", rpod(R(5, 1)), [rpod(R(5, 19))], A32, True)
fit_case(PFsrc + ":187", "equal edge case for init container", rpod(R(4, 1), init=[R(5, 1)]), [rpod(R(5, 19))], A32, True)
fit_case(PFsrc + ":193", "extended resource fits", rpod(R(scalar={EXT_A: 1})), [rpod(R())], A32, True)
fit_case(PFsrc + ":199", "extended resource fits for init container", rpod(R(), init=[R(scalar={EXT_A: 1})]),
         [rpod(R())], A32, True)
fit_case(PFsrc + ":205", "extended resource capacity enforced", rpod(R(1, 1, scalar={EXT_A: 10})),
         [rpod(R(0, 0, scalar={EXT_A: 0}))], A32, False, ["Insufficient " + EXT_A])
fit_case(PFsrc + ":214", "extended resource capacity enforced for init container",
         rpod(R(), init=[R(1, 1, scalar={EXT_A: 10})]), [rpod(R(0, 0, scalar={EXT_A: 0}))], A32, False,
         ["Insufficient " + EXT_A])
fit_case(PFsrc + ":223", "extended resource allocatable enforced", rpod(R(1, 1, scalar={EXT_A: 1})),
         [rpod(R(0, 0, scalar={EXT_A: 5}))], A32, False, ["Insufficient " + EXT_A])
fit_case(PFsrc + ":232", "extended resource allocatable enforced for init container",
         rpod(R(), init=[R(1, 1, scalar={EXT_A: 1})]), [rpod(R(0, 0, scalar={EXT_A: 5}))], A32, False,
         ["Insufficient " + EXT_A])
fit_case(PFsrc + ":241", "extended resource allocatable enforced for multiple containers",
         rpod(R(1, 1, scalar={EXT_A: 3}), R(1, 1, scalar={EXT_A: 3})), [rpod(R(0, 0, scalar={EXT_A: 2}))], A32, False,
         ["Insufficient " + EXT_A])
fit_case(PFsrc + ":251", "extended resource allocatable admits multiple init containers",
         rpod(R(), init=[R(1, 1, scalar={EXT_A: 3}), R(1, 1, scalar={EXT_A: 3})]), [rpod(R(0, 0, scalar={EXT_A: 2}))],
         A32, True)
fit_case(PFsrc + ":260", "extended resource allocatable enforced for multiple init containers",
         rpod(R(), init=[R(1, 1, scalar={EXT_A: 6}), R(1, 1, scalar={EXT_A: 3})]), [rpod(R(0, 0, scalar={EXT_A: 2}))],
         A32, False, ["Insufficient " + EXT_A])
fit_case(PFsrc + ":270", "extended resource allocatable enforced for unknown resource",
         rpod(R(1, 1, scalar={EXT_B: 1})), [rpod(R(0, 0))], A32, False, ["Insufficient " + EXT_B])
fit_case(PFsrc + ":279", "extended resource allocatable enforced for unknown resource for init container",
         rpod(R(), init=[R(1, 1, scalar={EXT_B: 1})]), [rpod(R(0, 0))], A32, False, ["Insufficient " + EXT_B])
fit_case(PFsrc + ":288", "hugepages resource capacity enforced", rpod(R(1, 1, scalar={HUGE_A: 10})),
         [rpod(R(0, 0, scalar={HUGE_A: 0}))], A32, False, ["Insufficient " + HUGE_A])
fit_case(PFsrc + ":297", "hugepages resource capacity enforced for init container",
         rpod(R(), init=[R(1, 1, scalar={HUGE_A: 10})]), [rpod(R(0, 0, scalar={HUGE_A: 0}))], A32, False,
         ["Insufficient " + HUGE_A])
fit_case(PFsrc + ":306", "hugepages resource allocatable enforced for multiple containers",
         rpod(R(1, 1, scalar={HUGE_A: 3}), R(1, 1, scalar={HUGE_A: 3})), [rpod(R(0, 0, scalar={HUGE_A: 2}))], A32, False,
         ["Insufficient " + HUGE_A])
# (:316 "skip checking ignored extended resource" needs extender-managed resources: out of scope)
A1 = alloc(10, 20, 0, 1, 0, 0, 0)
fit_case(PFsrc + ":349", "even without specified resources predicate fails when there's no space for additional pod",
         pod(), [rpod(R(10, 20))], A1, False, [IP])
fit_case(PFsrc + ":356", "even if both resources fit predicate fails when there's no space for additional pod",
         rpod(R(1, 1)), [rpod(R(5, 5))], A1, False, [IP])
fit_case(PFsrc + ":363", "even for equal edge case predicate fails when there's no space for additional pod",
         rpod(R(5, 1)), [rpod(R(5, 19))], A1, False, [IP])
fit_case(PFsrc + ":370", "even for equal edge case predicate fails when there's no space for additional pod due to init container",
         rpod(R(5, 1), init=[R(5, 1)]), [rpod(R(5, 19))], A1, False, [IP])
fit_case(PFsrc + ":401", "due to container scratch disk", rpod(R(1, 1)), [rpod(R(10, 10))], A32, False, [IC])
fit_case(PFsrc + ":410", "pod fit", rpod(R(1, 1)), [rpod(R(2, 10))], A32, True)
fit_case(PFsrc + ":416", "storage ephemeral local storage request exceeds allocatable", rpod(R(eph=25)),
         [rpod(R(2, 2))], A32, False, [IE])
fit_case(PFsrc + ":425", "pod fits", rpod(R(eph=10)), [rpod(R(2, 2))], A32, True)


# ------------------------------------------------ PodFitsHost
def pred_case(pred, src, test, p, n, fits, reasons, existing=()):
    ex = []
    for e in existing:
        e = json.loads(json.dumps(e))
        e["spec"]["nodeName"] = n["metadata"].get("name", "")
        ex.append(e)
    add("predicates", {"source": src, "test": test, "predicate": pred, "pod": p, "node": n,
                       "pods": ex, "fits": fits, "reasons": list(reasons) if not fits else []})


HN = "node(s) didn't match the requested hostname"
pred_case("HostName", PFsrc + ":478", "no host specified", pod(), node(""), True, [])
pred_case("HostName", PFsrc + ":484", "host matches", pod(node_name="foo"), node("foo"), True, [])
pred_case("HostName", PFsrc + ":497", "host doesn't match", pod(node_name="bar"), node("foo"), False, [HN])


# ------------------------------------------------ PodFitsHostPorts (predicates_test.go:533-667)
def ppod(*infos):
    ports = []
    for s in infos:
        proto, ip, port = s.split("/")
        ports.append({"hostIP": ip, "hostPort": int(port), "protocol": proto})
    return pod(node_name="m1", containers=[{"ports": ports}])


HP = "node(s) didn't have free ports for the requested pod ports"
for ln, test, want, have, fits in [
        (563, "nothing running", None, None, True),
        (569, "other port", ["UDP/127.0.0.1/8080"], ["UDP/127.0.0.1/9090"], True),
        (576, "same udp port", ["UDP/127.0.0.1/8080"], ["UDP/127.0.0.1/8080"], False),
        (583, "same tcp port", ["TCP/127.0.0.1/8080"], ["TCP/127.0.0.1/8080"], False),
        (590, "different host ip", ["TCP/127.0.0.1/8080"], ["TCP/127.0.0.2/8080"], True),
        (597, "different protocol", ["UDP/127.0.0.1/8080"], ["TCP/127.0.0.1/8080"], True),
        (604, "second udp port conflict", ["UDP/127.0.0.1/8000", "UDP/127.0.0.1/8080"], ["UDP/127.0.0.1/8080"], False),
        (611, "first tcp port conflict", ["TCP/127.0.0.1/8001", "UDP/127.0.0.1/8080"],
         ["TCP/127.0.0.1/8001", "UDP/127.0.0.1/8081"], False),
        (618, "first tcp port conflict due to 0.0.0.0 hostIP", ["TCP/0.0.0.0/8001"], ["TCP/127.0.0.1/8001"], False),
        (625, "TCP hostPort conflict due to 0.0.0.0 hostIP", ["TCP/10.0.10.10/8001", "TCP/0.0.0.0/8001"],
         ["TCP/127.0.0.1/8001"], False),
        (632, "second tcp port conflict to 0.0.0.0 hostIP", ["TCP/127.0.0.1/8001"], ["TCP/0.0.0.0/8001"], False),
        (639, "second different protocol", ["UDP/127.0.0.1/8001"], ["TCP/0.0.0.0/8001"], True),
        (646, "UDP hostPort conflict due to 0.0.0.0 hostIP", ["UDP/127.0.0.1/8001"],
         ["TCP/0.0.0.0/8001", "UDP/0.0.0.0/8001"], False)]:
    p = pod() if want is None else ppod(*want)
    ex = [] if have is None else [ppod(*have)]
    pred_case("PodFitsHostPorts", PFsrc + ":%d" % ln, test, p, node("m1"), fits, [HP], ex)

# ------------------------------------------------ PodMatchNodeSelector (predicates_test.go:894-1391)
NS = "node(s) didn't match node selector"


def req_aff(terms):
    return {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": terms}}}


def term(*exprs):
    return {"matchExpressions": list(exprs)}


for ln, test, p, labels, fits in [
        (901, "no selector", pod(), None, True),
        (906, "missing labels", pod(nodeSelector={"foo": "bar"}), None, False),
        (916, "same labels", pod(nodeSelector={"foo": "bar"}), {"foo": "bar"}, True),
        (929, "node labels are superset", pod(nodeSelector={"foo": "bar"}), {"foo": "bar", "baz": "blah"}, True),
        (943, "node labels are subset", pod(nodeSelector={"foo": "bar", "baz": "blah"}), {"foo": "bar"}, False),
        (957, "Pod with matchExpressions using In operator that matches the existing node",
         pod(affinity=req_aff([term(expr("foo", "In", ["bar", "value2"]))])), {"foo": "bar"}, True),
        (984, "Pod with matchExpressions using Gt operator that matches the existing node",
         pod(affinity=req_aff([term(expr("kernel-version", "Gt", ["0204"]))])), {"kernel-version": "0206"}, True),
        (1012, "Pod with matchExpressions using NotIn operator that matches the existing node",
         pod(affinity=req_aff([term(expr("mem-type", "NotIn", ["DDR", "DDR2"]))])), {"mem-type": "DDR3"}, True),
        (1039, "Pod with matchExpressions using Exists operator that matches the existing node",
         pod(affinity=req_aff([term(expr("GPU", "Exists"))])), {"GPU": "NVIDIA-GRID-K1"}, True),
        (1065, "Pod with affinity that don't match node's labels won't schedule onto the node",
         pod(affinity=req_aff([term(expr("foo", "In", ["value1", "value2"]))])), {"foo": "bar"}, False),
        (1092, "Pod with a nil []NodeSelectorTerm in affinity, can't match the node's labels and won't schedule onto the node",
         pod(affinity=req_aff(None)), {"foo": "bar"}, False),
        (1110, "Pod with an empty []NodeSelectorTerm in affinity, can't match the node's labels and won't schedule onto the node",
         pod(affinity=req_aff([])), {"foo": "bar"}, False),
        (1128, "Pod with empty MatchExpressions is not a valid value will match no objects and won't schedule onto the node",
         pod(affinity=req_aff([term()])), {"foo": "bar"}, False),
        (1146, "Pod with no Affinity will schedule onto a node", pod(), {"foo": "bar"}, True),
        (1153, "Pod with Affinity but nil NodeSelector will schedule onto a node",
         pod(affinity={"nodeAffinity": {}}), {"foo": "bar"}, True),
        (1169, "Pod with multiple matchExpressions ANDed that matches the existing node",
         pod(affinity=req_aff([term(expr("GPU", "Exists"), expr("GPU", "NotIn", ["AMD", "INTER"]))])),
         {"GPU": "NVIDIA-GRID-K1"}, True),
        (1200, "Pod with multiple matchExpressions ANDed that doesn't match the existing node",
         pod(affinity=req_aff([term(expr("GPU", "Exists"), expr("GPU", "In", ["AMD", "INTER"]))])),
         {"GPU": "NVIDIA-GRID-K1"}, False),
        (1231, "Pod with multiple NodeSelectorTerms ORed in affinity, matches the node's labels and will schedule onto the node",
         pod(affinity=req_aff([term(expr("foo", "In", ["bar", "value2"])), term(expr("diffkey", "In", ["wrong", "value2"]))])),
         {"foo": "bar"}, True),
        (1269, "Pod with an Affinity and a PodSpec.NodeSelector(the old thing that we are deprecating) both are satisfied, will schedule onto the node",
         pod(nodeSelector={"foo": "bar"}, affinity=req_aff([term(expr("foo", "Exists"))])), {"foo": "bar"}, True),
        (1300, "Pod with an Affinity matches node's labels but the PodSpec.NodeSelector(the old thing that we are deprecating) is not satisfied, won't schedule onto the node",
         pod(nodeSelector={"foo": "bar"}, affinity=req_aff([term(expr("foo", "Exists"))])), {"foo": "barrrrrr"}, False),
        (1331, "Pod with an invalid value in Affinity term won't be scheduled onto the node",
         pod(affinity=req_aff([term(expr("foo", "NotIn", ["invalid value: ___@#$%^"]))])), {"foo": "bar"}, False)]:
    if p["spec"].get("affinity", {}).get("nodeAffinity", {}).get("requiredDuringSchedulingIgnoredDuringExecution", {}) \
            and p["spec"]["affinity"]["nodeAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"].get("nodeSelectorTerms", 0) is None:
        p["spec"]["affinity"]["nodeAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"] = {}
    pred_case("MatchNodeSelector", PFsrc + ":%d" % ln, test, p, node("", labels=labels), fits, [NS])

# ------------------------------------------------ PodToleratesNodeTaints (predicates_test.go:3221-3422)
TX = "node(s) had taints that the pod didn't tolerate"
for ln, test, tols, taints, fits in [
        (3229, "a pod having no tolerations can't be scheduled onto a node with nonempty taints", None,
         [taint("dedicated", "user1", "NoSchedule")], False),
        (3243, "a pod which can be scheduled on a dedicated node assigned to user1 with effect NoSchedule",
         [{"key": "dedicated", "value": "user1", "effect": "NoSchedule"}], [taint("dedicated", "user1", "NoSchedule")], True),
        (3260, "a pod which can't be scheduled on a dedicated node assigned to user2 with effect NoSchedule",
         [tol("dedicated", "Equal", "user2", "NoSchedule")], [taint("dedicated", "user1", "NoSchedule")], False),
        (3277, "a pod can be scheduled onto the node, with a toleration uses operator Exists that tolerates the taints on the node",
         [{"key": "foo", "operator": "Exists", "effect": "NoSchedule"}], [taint("foo", "bar", "NoSchedule")], True),
        (3294, "a pod has multiple tolerations, node has multiple taints, all the taints are tolerated, pod can be scheduled onto the node",
         [tol("dedicated", "Equal", "user2", "NoSchedule"), {"key": "foo", "operator": "Exists", "effect": "NoSchedule"}],
         [taint("dedicated", "user2", "NoSchedule"), taint("foo", "bar", "NoSchedule")], True),
        (3317, "a pod has a toleration that keys and values match the taint on the node, but (non-empty) effect doesn't match, can't be scheduled onto the node",
         [tol("foo", "Equal", "bar", "PreferNoSchedule")], [taint("foo", "bar", "NoSchedule")], False),
        (3337, "The pod has a toleration that keys and values match the taint on the node, the effect of toleration is empty, and the effect of taint is NoSchedule. Pod can be scheduled onto the node",
         [tol("foo", "Equal", "bar", None)], [taint("foo", "bar", "NoSchedule")], True),
        (3357, "The pod has a toleration that key and value don't match the taint on the node, but the effect of taint on node is PreferNochedule. Pod can be scheduled onto the node",
         [tol("dedicated", "Equal", "user2", "NoSchedule")], [taint("dedicated", "user1", "PreferNoSchedule")], True),
        (3377, "The pod has no toleration, but the effect of taint on node is PreferNochedule. Pod can be scheduled onto the node",
         None, [taint("dedicated", "user1", "PreferNoSchedule")], True)]:
    p = pod(containers=[{"image": "img"}]) if tols is None else pod(containers=[{"image": "img"}], tolerations=tols)
    pred_case("PodToleratesNodeTaints", PFsrc + ":%d" % ln, test, p, node("", taints=taints), fits, [TX])

# ------------------------------------------------ memory / disk pressure (predicates_test.go:3428-3602)
be_pod = pod(containers=[{"name": "container", "image": "image", "resources": {}}])
nbe_pod = pod(containers=[{"name": "container", "image": "image",
                           "resources": {"requests": alloc(100, 100, 100, 100, 0, 0, 0)}}])
MP, DP = "node(s) had memory pressure", "node(s) had disk pressure"
no_mp = node("", conditions=[("Ready", "True")])
mp = node("", conditions=[("MemoryPressure", "True")])
for ln, test, p, n, fits in [
        (3479, "best-effort pod schedulable on node without memory pressure condition on", be_pod, no_mp, True),
        (3485, "best-effort pod not schedulable on node with memory pressure condition on", be_pod, mp, False),
        (3491, "non best-effort pod schedulable on node with memory pressure condition on", nbe_pod, mp, True),
        (3497, "non best-effort pod schedulable on node without memory pressure condition on", nbe_pod, no_mp, True)]:
    pred_case("CheckNodeMemoryPressure", PFsrc + ":%d" % ln, test, p, n, fits, [MP])
dp = node("", conditions=[("DiskPressure", "True")])
no_dp = node("", conditions=[("Ready", "True")])
simple = pod(containers=[{"name": "container", "image": "image", "imagePullPolicy": "Always"}])
pred_case("CheckNodeDiskPressure", PFsrc + ":3574", "pod schedulable on node without pressure condition on", simple, no_dp, True, [DP])
pred_case("CheckNodeDiskPressure", PFsrc + ":3580", "pod not schedulable on node with pressure condition on", simple, dp, False, [DP])

# ------------------------------------------------ CheckNodeCondition (predicates_test.go:3604-3676)
for i, (conds, unsched, ok) in enumerate([
        ([("Ready", "True")], None, True), ([("Ready", "False")], None, False), ([("OutOfDisk", "True")], None, False),
        ([("OutOfDisk", "False")], None, True), ([("Ready", "True"), ("OutOfDisk", "True")], None, False),
        ([("Ready", "True"), ("OutOfDisk", "False")], None, True), ([("Ready", "False"), ("OutOfDisk", "True")], None, False),
        ([("Ready", "False"), ("OutOfDisk", "False")], None, False), (None, True, False), (None, False, True),
        (None, None, True)]):
    n = node("node%d" % (i + 1), conditions=conds, unschedulable=unsched)
    add("predicates", {"source": PFsrc + ":%d" % (3611 + 5 * i), "test": "node%d" % (i + 1),
                       "predicate": "CheckNodeCondition", "pod": pod(), "node": n, "pods": [], "fits": ok,
                       "reasons": None})

# ------------------------------------------------ NodeInfo.AddPod (schedulercache/node_info_test.go:449-600)
ni_pods = [pod(name="test-1", node_name="test-node", containers=[
    {"resources": {"requests": {"cpu": "100m", "memory": "500"}},
     "ports": [{"hostIP": "127.0.0.1", "hostPort": 80, "protocol": "TCP"}]}]),
    pod(name="test-2", node_name="test-node", containers=[
        {"resources": {"requests": {"cpu": "200m", "memory": "1Ki"}},
         "ports": [{"hostIP": "127.0.0.1", "hostPort": 8080, "protocol": "TCP"}]}])]
add("node_info", {"source": S + "schedulercache/node_info_test.go:449", "test": "TestNodeInfoAddPod",
                  "node": node("test-node"), "pods": ni_pods,
                  "expect": {"requested_cpu": 300, "requested_mem": 1524, "nonzero_cpu": 300, "nonzero_mem": 1524,
                             "pod_count": 2,
                             "used_ports": [["127.0.0.1", "TCP", 80], ["127.0.0.1", "TCP", 8080]]}})

# ------------------------------------------------ TestZeroRequest (core/generic_scheduler_test.go:534-660)
DM, DC = 200 * 1024 * 1024, 100
zr_none = {"containers": [{}]}


def zpod(spec, nn=None):
    p = {"metadata": {}, "spec": json.loads(json.dumps(spec))}
    if nn:
        p["spec"]["nodeName"] = nn
    return p


small = {"containers": [ctr("%dm" % DC, "%d" % DM)]}
large = {"containers": [ctr("%dm" % (DC * 3), "%d" % (DM * 3))]}
zr_nodes = [node("machine1", 1000, DM * 10, pods=100), node("machine2", 1000, DM * 10, pods=100)]
zr_pods = [zpod(large, "machine1"), zpod(zr_none, "machine1"), zpod(large, "machine2"), zpod(small, "machine2")]
ZRsrc = S + "core/generic_scheduler_test.go"
for ln, test, p, eq in [
        (577, "test priority of zero-request pod with machine with zero-request pod", zpod(zr_none), True),
        (587, "test priority of nonzero-request pod with machine with zero-request pod", zpod(small), True),
        (598, "test priority of larger pod with machine with zero-request pod", zpod(large), False)]:
    add("prioritize", {"source": ZRsrc + ":%d" % ln, "test": test, "pod": p, "nodes": zr_nodes, "pods": zr_pods,
                       "configs": [["LeastRequestedPriority", 1], ["BalancedResourceAllocation", 1],
                                   ["SelectorSpreadPriority", 1]],
                       "expect_all_equal" if eq else "expect_none_equal": 25})

# ------------------------------------------------ TestSelectHost (core/generic_scheduler_test.go:121-185)
for ln, lst, possible in [
        (129, [["machine1.1", 1], ["machine2.1", 2]], ["machine2.1"]),
        (137, [["machine1.1", 1], ["machine1.2", 2], ["machine1.3", 2], ["machine2.1", 2]],
         ["machine1.2", "machine1.3", "machine2.1"]),
        (147, [["machine1.1", 3], ["machine1.2", 3], ["machine2.1", 2], ["machine3.1", 1], ["machine1.3", 3]],
         ["machine1.1", "machine1.2", "machine1.3"])]:
    add("select_host", {"source": ZRsrc + ":%d" % ln, "list": lst, "possible": possible, "calls": 10})

# ------------------------------------------------ TestHumanReadableFitError (core/generic_scheduler_test.go:508-523)
add("fit_error", {"source": ZRsrc + ":508", "num_nodes": 3,
                  "failed": {"1": ["node(s) had memory pressure"], "2": ["node(s) had disk pressure"],
                             "3": ["node(s) had disk pressure"]},
                  "contains": ["0/3 nodes are available", "2 node(s) had disk pressure", "1 node(s) had memory pressure"]})

# ------------------------------------------------ Quantity → int64 (AM/pkg/api/resource/quantity.go:695-713;
# expected values follow the documented ceil semantics and the fixtures the scheduler tests rely on)
for s, milli, val in [("1", 1000, 1), ("100m", 100, 1), ("1000m", 1000, 1), ("2000", 2000000, 2000),
                      ("1Ki", 1024000, 1024), ("128Mi", 134217728000, 134217728), ("1Gi", 1073741824000, 1073741824),
                      ("0.1", 100, 1), ("1.5", 1500, 2), ("0", 0, 0), ("1e3", 1000000, 1000), ("1k", 1000000, 1000),
                      ("0.0001", 1, 1), ("250m", 250, 1), ("209715200", 209715200000, 209715200)]:
    add("quantity", {"source": "vendor/k8s.io/apimachinery/pkg/api/resource/quantity.go:695", "q": s,
                     "milli": milli, "value": val})

# ------------------------------------------------ Policy decoding (algorithmprovider/defaults/compatibility_test.go)
CT = "vendor/k8s.io/kubernetes/pkg/scheduler/algorithmprovider/defaults/compatibility_test.go"
SA = {"serviceAffinity": {"labels": ["region"]}}
LP = {"labelsPresence": {"labels": ["foo"], "presence": True}}
SAA = {"serviceAntiAffinity": {"label": "zone"}}
LPR = {"labelPreference": {"label": "bar", "presence": True}}
for ver, ln, preds, prios in [
        ("1.0", 49, [["MatchNodeSelector", None], ["PodFitsResources", None], ["PodFitsPorts", None],
                     ["NoDiskConflict", None], ["TestServiceAffinity", SA], ["TestLabelsPresence", LP]],
         [["LeastRequestedPriority", 1, None], ["ServiceSpreadingPriority", 2, None],
          ["TestServiceAntiAffinity", 3, SAA], ["TestLabelPreference", 4, LPR]]),
        ("1.1", 87, [["MatchNodeSelector", None], ["PodFitsHostPorts", None], ["PodFitsResources", None],
                     ["NoDiskConflict", None], ["HostName", None], ["TestServiceAffinity", SA],
                     ["TestLabelsPresence", LP]],
         [["EqualPriority", 2, None], ["LeastRequestedPriority", 2, None], ["BalancedResourceAllocation", 2, None],
          ["SelectorSpreadPriority", 2, None], ["TestServiceAntiAffinity", 3, SAA], ["TestLabelPreference", 4, LPR]]),
        ("1.9", 460, [[n, None] for n in ["MatchNodeSelector", "PodFitsResources", "PodFitsHostPorts", "HostName",
                                          "NoDiskConflict", "NoVolumeZoneConflict", "PodToleratesNodeTaints",
                                          "CheckNodeMemoryPressure", "CheckNodeDiskPressure", "CheckNodeCondition",
                                          "MaxEBSVolumeCount", "MaxGCEPDVolumeCount", "MaxAzureDiskVolumeCount",
                                          "MatchInterPodAffinity", "GeneralPredicates", "CheckVolumeBinding"]]
         + [["TestServiceAffinity", SA], ["TestLabelsPresence", LP]],
         [[n, 2, None] for n in ["EqualPriority", "ImageLocalityPriority", "LeastRequestedPriority",
                                 "BalancedResourceAllocation", "SelectorSpreadPriority", "NodePreferAvoidPodsPriority",
                                 "NodeAffinityPriority", "TaintTolerationPriority", "InterPodAffinityPriority",
                                 "MostRequestedPriority"]])]:
    doc = {"kind": "Policy", "apiVersion": "v1",
           "predicates": [dict({"name": n}, **({"argument": a} if a else {})) for n, a in preds],
           "priorities": [dict({"name": n, "weight": w}, **({"argument": a} if a else {})) for n, w, a in prios]}
    add("policy", {"source": CT + ":%d" % ln, "version": ver, "json": json.dumps(doc),
                   "predicates": preds, "priorities": prios})

# ------------------------------------------------ ValidatePolicy (api/validation/validation_test.go:27-86)
VT = "vendor/k8s.io/kubernetes/pkg/scheduler/api/validation/validation_test.go"
MAXW = ((1 << 63) - 1) // 10
for ln, pol, err in [
        (33, {"priorities": [{"name": "NoWeightPriority"}]},
         "Priority NoWeightPriority should have a positive weight applied to it or it has overflown"),
        (37, {"priorities": [{"name": "NoWeightPriority", "weight": 0}]},
         "Priority NoWeightPriority should have a positive weight applied to it or it has overflown"),
        (41, {"priorities": [{"name": "WeightPriority", "weight": 2}]}, None),
        (45, {"priorities": [{"name": "WeightPriority", "weight": -2}]},
         "Priority WeightPriority should have a positive weight applied to it or it has overflown"),
        (49, {"priorities": [{"name": "WeightPriority", "weight": MAXW}]},
         "Priority WeightPriority should have a positive weight applied to it or it has overflown"),
        (53, {"extenders": [{"urlPrefix": "http://127.0.0.1:8081/extender", "prioritizeVerb": "prioritize",
                             "weight": 2}]}, None),
        (57, {"extenders": [{"urlPrefix": "http://127.0.0.1:8081/extender", "prioritizeVerb": "prioritize",
                             "weight": -2}]},
         "Priority for extender http://127.0.0.1:8081/extender should have a positive weight applied to it"),
        (61, {"extenders": [{"urlPrefix": "http://127.0.0.1:8081/extender", "filterVerb": "filter"}]}, None),
        (65, {"extenders": [{"urlPrefix": "http://127.0.0.1:8081/extender", "bindVerb": "bind"},
                            {"urlPrefix": "http://127.0.0.1:8082/extender", "bindVerb": "bind"}]},
         "Only one extender can implement bind, found 2"),
        (72, {"extenders": [{"urlPrefix": "http://127.0.0.1:8081/extender", "managedResources": [{"name": "foo.com/bar"}]},
                            {"urlPrefix": "http://127.0.0.1:8082/extender", "bindVerb": "bind",
                             "managedResources": [{"name": "foo.com/bar"}]}]},
         "Duplicate extender managed resource name foo.com/bar"),
        (80, {"extenders": [{"urlPrefix": "http://127.0.0.1:8081/extender",
                             "managedResources": [{"name": "kubernetes.io/foo"}]}]},
         "kubernetes.io/foo is an invalid extended resource name")]:
    add("policy_validation", {"source": VT + ":%d" % ln, "policy": pol, "error": err})


# ------------------------------------------------ inter-pod affinity (predicate + priority)
# The cases of TestInterPodAffinity / TestInterPodAffinityWithMultipleNodes
# (S/algorithm/predicates/predicates_test.go:2168-3146) and TestInterPodAffinityPriority /
# TestHardPodAffinitySymmetricWeight (S/algorithm/priorities/interpod_affinity_test.go:42-615)
# are long struct literals: they are read from the reference test files by go_literal.py (data
# only) rather than retyped.  Each case keeps its harness semantics:
#  - predicate, single node: every test pod is listed by the pod lister, and FakeNodeInfo maps
#    any node name to the test node; the metadata sees only the pods on that node;
#  - predicate, multiple nodes: pods resolve to their own node (FakeNodeListInfo); the metadata
#    sees the pods of the node under test, or is absent ("nometa": computed from every pod);
#  - priority: every node's pods (CreateNodeNameToInfoMap), hard weight 1 (the Go default) or
#    the case's hardPodAffinityWeight.
REF = "/root/reference/"
IPA_REASONS = {"ErrPodAffinityNotMatch": "node(s) didn't match pod affinity/anti-affinity",
               "ErrPodAffinityRulesNotMatch": "node(s) didn't match pod affinity rules",
               "ErrPodAntiAffinityRulesNotMatch": "node(s) didn't match pod anti-affinity rules",
               "ErrExistingPodsAntiAffinityRulesNotMatch": "node(s) didn't satisfy existing pods anti-affinity rules"}


def _line_of(src, text, start):
    i = src.find('"%s' % text[:40].replace('"', '\\"'), start)
    return src.count("\n", 0, i) + 1 if i >= 0 else 0


def _reasons(lst):
    return [IPA_REASONS[r["__ident__"]] for r in (lst or [])]


def interpod_cases():
    import go_literal as g
    pf = S + "algorithm/predicates/predicates_test.go"
    with open(REF + pf) as f:
        src = f.read()
    start = src.index("func TestInterPodAffinity(")
    _, cs = g.parse_test(src, "TestInterPodAffinity")
    for c in cs:
        add("interpod_predicates", {"source": "%s:%d" % (pf, _line_of(src, c["test"], start)), "test": c["test"],
                                    "pod": c["pod"], "pods": c.get("pods") or [], "nodes": [c["node"]],
                                    "single_node": True, "nometa": False,
                                    "fits": {c["node"]["metadata"]["name"]: c["fits"]},
                                    "reasons": {c["node"]["metadata"]["name"]: _reasons(c.get("expectFailureReasons"))}})
    start = src.index("func TestInterPodAffinityWithMultipleNodes(")
    _, cs = g.parse_test(src, "TestInterPodAffinityWithMultipleNodes")
    for c in cs:
        names = [n["metadata"]["name"] for n in c["nodes"]]
        exp = c.get("nodesExpectAffinityFailureReasons") or [None] * len(names)
        add("interpod_predicates", {"source": "%s:%d" % (pf, _line_of(src, c["test"], start)), "test": c["test"],
                                    "pod": c["pod"], "pods": c.get("pods") or [], "nodes": c["nodes"],
                                    "single_node": False, "nometa": bool(c.get("nometa")), "fits": c["fits"],
                                    "reasons": {n: _reasons(r) for n, r in zip(names, exp)}})
    qf = S + "algorithm/priorities/interpod_affinity_test.go"
    with open(REF + qf) as f:
        src = f.read()
    for fn, hw in (("TestInterPodAffinityPriority", 1), ("TestHardPodAffinitySymmetricWeight", None)):
        start = src.index("func %s(" % fn)
        _, cs = g.parse_test(src, fn)
        for c in cs:
            add("interpod_priorities", {"source": "%s:%d" % (qf, _line_of(src, c["test"], start)), "test": c["test"],
                                        "pod": c["pod"], "pods": c.get("pods") or [], "nodes": c["nodes"],
                                        "hard_weight": c["hardPodAffinityWeight"] if hw is None else hw,
                                        "expect": {h["host"]: h["score"] for h in c["expectedList"]}})



# ------------------------------------------------ volumes (predicates_test.go:669-891, 1622-2039, 3676-3913)
def vpod(vols, ns=None, name=None):
    md = {}
    if ns is not None:
        md["namespace"] = ns
    if name is not None:
        md["name"] = name
    return {"metadata": md, "spec": {"volumes": vols}}


def vol_case(pred, src, test, p, existing, fits, reasons, node=None, pvs=(), pvcs=(), max_vols=None):
    n = node if node is not None else {"metadata": {"name": "node"}}
    ex = []
    for k, e in enumerate(existing):
        e = json.loads(json.dumps(e))
        e["metadata"].setdefault("name", "existing-%d" % k)
        e["spec"]["nodeName"] = n["metadata"].get("name", "")
        ex.append(e)
    add("volumes", {"source": src, "test": test, "predicate": pred, "pod": p, "node": n, "pods": ex,
                    "pvs": list(pvs), "pvcs": list(pvcs), "max_vols": max_vols, "fits": fits,
                    "reasons": list(reasons) if not fits else []})


PT = S + "algorithm/predicates/predicates_test.go"
DC = "node(s) had no available disk"
for fn, line, k, field, a, b in (
        ("TestGCEDiskConflicts", 669, "gcePersistentDisk", "pdName", "foo", "bar"),
        ("TestAWSDiskConflicts", 722, "awsElasticBlockStore", "volumeID", "foo", "bar"),
        ("TestISCSIDiskConflicts", 834, "iscsi", "iqn", "iqn.2016-12.server:storage.target01",
         "iqn.2017-12.server:storage.target01")):
    extra = {"targetPortal": "127.0.0.1:3260", "fsType": "ext4", "lun": 0} if k == "iscsi" else {}
    vs1 = [{k: dict(extra, **{field: a})}]
    vs2 = [{k: dict(extra, **{field: b})}]
    base = line + 29 if k != "iscsi" else line + 35
    vol_case("NoDiskConflict", "%s:%d" % (PT, base), fn + " nothing", vpod([]), [], True, [])
    vol_case("NoDiskConflict", "%s:%d" % (PT, base + 1), fn + " one state", vpod([]), [vpod(vs1)], True, [])
    vol_case("NoDiskConflict", "%s:%d" % (PT, base + 2), fn + " same state", vpod(vs1), [vpod(vs1)], False, [DC])
    vol_case("NoDiskConflict", "%s:%d" % (PT, base + 3), fn + " different state", vpod(vs2), [vpod(vs1)], True, [])
rbd1 = [{"rbd": {"monitors": ["a", "b"], "pool": "foo", "image": "bar", "fsType": "ext4"}}]
rbd2 = [{"rbd": {"monitors": ["c", "d"], "pool": "foo", "image": "bar", "fsType": "ext4"}}]
vol_case("NoDiskConflict", PT + ":810", "TestRBDDiskConflicts nothing", vpod([]), [], True, [])
vol_case("NoDiskConflict", PT + ":811", "TestRBDDiskConflicts one state", vpod([]), [vpod(rbd1)], True, [])
vol_case("NoDiskConflict", PT + ":812", "TestRBDDiskConflicts same state", vpod(rbd1), [vpod(rbd1)], False, [DC])
vol_case("NoDiskConflict", PT + ":813", "TestRBDDiskConflicts different state", vpod(rbd2), [vpod(rbd1)], True, [])

# TestEBSVolumeCountConflicts (:1622-2039): pods :1623-1828, fake listers :1979-2021
ebs = lambda i: {"awsElasticBlockStore": {"volumeID": i}}
pvc = lambda c: {"persistentVolumeClaim": {"claimName": c}}
hostpath = {"hostPath": {}}
EV = {"oneVolPod": vpod([ebs("ovp")]), "ebsPVCPod": vpod([pvc("someEBSVol")]),
      "splitPVCPod": vpod([pvc("someNonEBSVol"), pvc("someEBSVol")]), "twoVolPod": vpod([ebs("tvp1"), ebs("tvp2")]),
      "splitVolsPod": vpod([hostpath, ebs("svp")]), "nonApplicablePod": vpod([hostpath]),
      "deletedPVCPod": vpod([pvc("deletedPVC")]), "twoDeletedPVCPod": vpod([pvc("deletedPVC"), pvc("anotherDeletedPVC")]),
      "deletedPVPod": vpod([pvc("pvcWithDeletedPV")]), "deletedPVPod2": vpod([pvc("pvcWithDeletedPV")]),
      "anotherDeletedPVPod": vpod([pvc("anotherPVCWithDeletedPV")]), "emptyPod": vpod([]),
      "unboundPVCPod": vpod([pvc("unboundPVC")]), "unboundPVCPod2": vpod([pvc("unboundPVC")]),
      "anotherUnboundPVCPod": vpod([pvc("anotherUnboundPVC")])}
EBS_PVS = [{"metadata": {"name": "someEBSVol"}, "spec": {"awsElasticBlockStore": {"volumeID": "ebsVol"}}},
           {"metadata": {"name": "someNonEBSVol"}, "spec": {}}]
EBS_PVCS = [{"metadata": {"name": n}, "spec": {"volumeName": v}} for n, v in (
    ("someEBSVol", "someEBSVol"), ("someNonEBSVol", "someNonEBSVol"), ("pvcWithDeletedPV", "pvcWithDeletedPV"),
    ("anotherPVCWithDeletedPV", "anotherPVCWithDeletedPV"), ("unboundPVC", ""), ("anotherUnboundPVC", ""))]
MV = "node(s) exceed max volume count"
for line, new, existing, mv, fits, test in (
        (1837, "oneVolPod", ["twoVolPod", "oneVolPod"], 4, True, "fits when node capacity >= new pod's EBS volumes"),
        (1844, "twoVolPod", ["oneVolPod"], 2, False, "doesn't fit when node capacity < new pod's EBS volumes"),
        (1851, "splitVolsPod", ["twoVolPod"], 3, True, "new pod's count ignores non-EBS volumes"),
        (1858, "twoVolPod", ["splitVolsPod", "nonApplicablePod", "emptyPod"], 3, True,
         "existing pods' counts ignore non-EBS volumes"),
        (1865, "ebsPVCPod", ["splitVolsPod", "nonApplicablePod", "emptyPod"], 3, True,
         "new pod's count considers PVCs backed by EBS volumes"),
        (1872, "splitPVCPod", ["splitVolsPod", "oneVolPod"], 3, True, "new pod's count ignores PVCs not backed by EBS volumes"),
        (1879, "twoVolPod", ["oneVolPod", "ebsPVCPod"], 3, False, "existing pods' counts considers PVCs backed by EBS volumes"),
        (1886, "twoVolPod", ["oneVolPod", "twoVolPod", "ebsPVCPod"], 4, True, "already-mounted EBS volumes are always ok to allow"),
        (1893, "splitVolsPod", ["oneVolPod", "oneVolPod", "ebsPVCPod"], 3, True, "the same EBS volumes are not counted multiple times"),
        (1900, "ebsPVCPod", ["oneVolPod", "deletedPVCPod"], 2, False, "pod with missing PVC is counted towards the PV limit"),
        (1907, "ebsPVCPod", ["oneVolPod", "deletedPVCPod"], 3, True, "pod with missing PVC is counted towards the PV limit"),
        (1914, "ebsPVCPod", ["oneVolPod", "twoDeletedPVCPod"], 3, False, "pod with missing two PVCs is counted towards the PV limit twice"),
        (1921, "ebsPVCPod", ["oneVolPod", "deletedPVPod"], 2, False, "pod with missing PV is counted towards the PV limit"),
        (1928, "ebsPVCPod", ["oneVolPod", "deletedPVPod"], 3, True, "pod with missing PV is counted towards the PV limit"),
        (1935, "deletedPVPod2", ["oneVolPod", "deletedPVPod"], 2, True,
         "two pods missing the same PV are counted towards the PV limit only once"),
        (1942, "anotherDeletedPVPod", ["oneVolPod", "deletedPVPod"], 2, False,
         "two pods missing different PVs are counted towards the PV limit twice"),
        (1949, "ebsPVCPod", ["oneVolPod", "unboundPVCPod"], 2, False, "pod with unbound PVC is counted towards the PV limit"),
        (1956, "ebsPVCPod", ["oneVolPod", "unboundPVCPod"], 3, True, "pod with unbound PVC is counted towards the PV limit"),
        (1963, "unboundPVCPod2", ["oneVolPod", "unboundPVCPod"], 2, True,
         "the same unbound PVC in multiple pods is counted towards the PV limit only once"),
        (1970, "anotherUnboundPVCPod", ["oneVolPod", "unboundPVCPod"], 2, False,
         "two different unbound PVCs are counted towards the PV limit as two volumes")):
    vol_case("MaxEBSVolumeCount", "%s:%d" % (PT, line), test, EV[new], [EV[e] for e in existing], fits, [MV],
             pvs=EBS_PVS, pvcs=EBS_PVCS, max_vols=mv)

# TestVolumeZonePredicate / ...MultiZone (:3694-3913); createPodWithVolume :3676-3692
ZK, RK = "failure-domain.beta.kubernetes.io/zone", "failure-domain.beta.kubernetes.io/region"
VZ = "node(s) had no available volume zone"
zpvcs = [{"metadata": {"name": "PVC_%d" % i, "namespace": "default"}, "spec": {"volumeName": v}}
         for i, v in ((1, "Vol_1"), (2, "Vol_2"), (3, "Vol_3"), (4, "Vol_not_exist"))]
cpv = lambda pod_name, pv, c: {"metadata": {"name": pod_name, "namespace": "default"},
                               "spec": {"volumes": [{"name": pv, "persistentVolumeClaim": {"claimName": c}}]}}
znode = lambda labels: {"metadata": dict({"name": "host1"}, **({"labels": labels} if labels else {}))}
zpvs1 = [{"metadata": {"name": "Vol_1", "labels": {ZK: "us-west1-a"}}},
         {"metadata": {"name": "Vol_2", "labels": {RK: "us-west1-b", "uselessLabel": "none"}}},
         {"metadata": {"name": "Vol_3", "labels": {RK: "us-west1-c"}}}]
for line, test, p, labels, fits in (
        (3732, "pod without volume", {"metadata": {"name": "pod_1", "namespace": "default"}, "spec": {}}, {ZK: "us-west1-a"}, True),
        (3745, "node without labels", cpv("pod_1", "vol_1", "PVC_1"), None, True),
        (3755, "label zone failure domain matched", cpv("pod_1", "vol_1", "PVC_1"), {ZK: "us-west1-a", "uselessLabel": "none"}, True),
        (3766, "label zone region matched", cpv("pod_1", "vol_1", "PVC_2"), {RK: "us-west1-b", "uselessLabel": "none"}, True),
        (3777, "label zone region failed match", cpv("pod_1", "vol_1", "PVC_2"), {RK: "no_us-west1-b", "uselessLabel": "none"}, False),
        (3788, "label zone failure domain failed match", cpv("pod_1", "vol_1", "PVC_1"),
         {ZK: "no_us-west1-a", "uselessLabel": "none"}, False)):
    vol_case("NoVolumeZoneConflict", "%s:%d" % (PT, line), test, p, [], fits, [VZ], node=znode(labels), pvs=zpvs1,
             pvcs=zpvcs)
zpvs2 = [{"metadata": {"name": "Vol_1", "labels": {ZK: "us-west1-a"}}},
         {"metadata": {"name": "Vol_2", "labels": {ZK: "us-west1-b", "uselessLabel": "none"}}},
         {"metadata": {"name": "Vol_3", "labels": {ZK: "us-west1-c__us-west1-a"}}}]
for line, test, p, labels, fits in (
        (3860, "multi-zone node without labels", cpv("pod_1", "Vol_3", "PVC_3"), None, True),
        (3870, "multi-zone label zone failure domain matched", cpv("pod_1", "Vol_3", "PVC_3"),
         {ZK: "us-west1-a", "uselessLabel": "none"}, True),
        (3881, "multi-zone label zone failure domain failed match", cpv("pod_1", "vol_1", "PVC_1"),
         {ZK: "us-west1-b", "uselessLabel": "none"}, False)):
    vol_case("NoVolumeZoneConflict", "%s:%d" % (PT, line), test, p, [], fits, [VZ], node=znode(labels), pvs=zpvs2,
             pvcs=zpvcs)


def spread_cases():
    """TestSelectorSpreadPriority / TestZoneSelectorSpreadPriority (selector_spreading_test.go:43-366,
    375-812): services / RCs / RSs / StatefulSets selecting the pod, placed pods, expected scores."""
    import go_literal as g
    sf = S + "algorithm/priorities/selector_spreading_test.go"
    with open(REF + sf) as f:
        src = f.read()
    zone_nodes = {"nodeMachine1Zone1": ("machine1.zone1", "zone1"), "nodeMachine1Zone2": ("machine1.zone2", "zone2"),
                  "nodeMachine2Zone2": ("machine2.zone2", "zone2"), "nodeMachine1Zone3": ("machine1.zone3", "zone3"),
                  "nodeMachine2Zone3": ("machine2.zone3", "zone3"), "nodeMachine3Zone3": ("machine3.zone3", "zone3")}
    consts = {"metav1.NamespaceDefault": "default"}
    consts.update({k: v[0] for k, v in zone_nodes.items()})

    def res(x):
        if isinstance(x, dict):
            if "__ident__" in x:
                return consts[x["__ident__"]]
            if x.get("__call__") == "buildPod":
                nn, lab, _ = (res(a) for a in x["args"])
                pod = {"metadata": {"labels": lab or {}}, "spec": {}}
                if nn:
                    pod["spec"]["nodeName"] = nn
                return pod
            if x.get("__call__") == "new":
                return {}
            if x.get("__call__") == "controllerRef":
                return None      # owner references play no part in getSelectors
            if "__call__" in x:
                raise ValueError(x)
            return {k: res(v) for k, v in x.items()}
        if isinstance(x, list):
            return [res(v) for v in x]
        return x
    for fn in ("TestSelectorSpreadPriority", "TestZoneSelectorSpreadPriority"):
        start = src.index("func %s(" % fn)
        _, cs = g.parse_test(src, fn)
        for c in cs:
            c = res(c)
            pod = c.get("pod") or {}
            pod.setdefault("metadata", {})
            if fn == "TestZoneSelectorSpreadPriority":
                nodes = [{"metadata": {"name": nm, "labels": {"failure-domain.beta.kubernetes.io/zone": z}}}
                         for nm, z in zone_nodes.values()]
            else:
                nodes = [{"metadata": {"name": nm}} for nm in c["nodes"]]
            add("spread", {"source": "%s:%d" % (sf, _line_of(src, c["test"], start)), "test": c["test"],
                           "pod": pod, "pods": c.get("pods") or [], "nodes": nodes,
                           "services": c.get("services") or [], "rcs": c.get("rcs") or [], "rss": c.get("rss") or [],
                           "sss": c.get("sss") or [],
                           "expect": {h["host"]: h["score"] for h in c["expectedList"]}})

def label_priority_cases():
    """TestNewNodeLabelPriority (node_label_test.go:30-128) and TestZoneSpreadPriority — the
    ServiceAntiAffinity priority with label "zone" (selector_spreading_test.go:605-760)."""
    import go_literal as g
    nf = S + "algorithm/priorities/node_label_test.go"
    with open(REF + nf) as f:
        src = f.read()
    start = src.index("func TestNewNodeLabelPriority(")
    _, cs = g.parse_test(src, "TestNewNodeLabelPriority")
    for c in cs:
        add("label_priorities", {"source": "%s:%d" % (nf, _line_of(src, c["test"], start)), "test": c["test"],
                                 "kind": "labelPreference", "label": c["label"], "presence": c["presence"],
                                 "pod": {"metadata": {}}, "pods": [], "nodes": c["nodes"], "services": [],
                                 "expect": {h["host"]: h["score"] for h in c["expectedList"]}})
    sf = S + "algorithm/priorities/selector_spreading_test.go"
    with open(REF + sf) as f:
        src = f.read()
    start = src.index("func TestZoneSpreadPriority(")
    _, cs = g.parse_test(src, "TestZoneSpreadPriority")
    for c in cs:
        pod = c.get("pod") or {}
        if pod.get("__call__") == "new":
            pod = {}
        pod.setdefault("metadata", {})
        nodes = [{"metadata": {"name": nm, "labels": lab}} for nm, lab in c["nodes"].items()]
        add("label_priorities", {"source": "%s:%d" % (sf, _line_of(src, c["test"], start)), "test": c["test"],
                                 "kind": "serviceAntiAffinity", "label": "zone", "pod": pod,
                                 "pods": c.get("pods") or [], "nodes": nodes, "services": c.get("services") or [],
                                 "expect": {h["host"]: h["score"] for h in c["expectedList"]}})


def service_affinity_cases():
    """TestServiceAffinity (predicates_test.go:1460-1620): the pod lister's pods, the service
    lister's services, the node list of the five machines; the predicate's NodeInfo holds the test
    node and no pods."""
    import go_literal as g
    pf = S + "algorithm/predicates/predicates_test.go"
    with open(REF + pf) as f:
        src = f.read()
    start = src.index("func TestServiceAffinity(")
    loc, cs = g.parse_test(src, "TestServiceAffinity")
    nodes = [loc["node%d" % i] for i in range(1, 6)]
    for c in cs:
        add("service_affinity", {"source": "%s:%d" % (pf, _line_of(src, c["test"], start)), "test": c["test"],
                                 "pod": c.get("pod") or {"metadata": {}}, "pods": c.get("pods") or [],
                                 "node": c["node"], "nodes": nodes, "services": c.get("services") or [],
                                 "labels": c["labels"], "fits": c["fits"]})


if os.path.isdir(REF):
    interpod_cases()
    spread_cases()
    label_priority_cases()
    service_affinity_cases()
else:  # keep the committed fixtures when the reference checkout is absent
    for group in ("interpod_predicates", "interpod_priorities", "spread", "label_priorities", "service_affinity"):
        with open(os.path.join(HERE, group + ".json")) as f:
            cases[group] = json.load(f)

if __name__ == "__main__":
    for group, lst in cases.items():
        with open(os.path.join(HERE, group + ".json"), "w") as f:
            json.dump(lst, f, indent=1, sort_keys=True)
        print(group, len(lst))
