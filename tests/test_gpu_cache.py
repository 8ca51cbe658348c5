"""Per-pod drop-in parity (GPU): the scheduleOne loop through both cache mirrors —
ksim.cache.SchedulerCache (Python host over ksim_schedule_one + the cache-event entry points of
include/ksim.h) and ksim.frontend.K8sCache (the C++ scheduler cache of include/ksim_k8s.h, what a cgo
adapter drives: every rule in the library) — against the object-level oracle's SchedulerCache
(oracle/ksim_ref.py, restating schedulercache/cache.go and genericScheduler.Schedule), on seeded
streams that interleave Schedule + assume with node add / update / remove and pod add / confirm /
update / remove / forget events.  Every decision (host or FitError text), lastNodeIndex and the
final per-node state must be identical."""
import ctypes as C

import pytest

import ksim_ref as R
from events import apply, event_stream
from ksim import abi, scheduler
from ksim.cache import SchedulerCache
from ksim.frontend import K8sCache

pytestmark = pytest.mark.gpu


class K8sCacheAdapter(K8sCache):
    """The C++ cache driven the way the cgo adapter in INTEGRATION.md drives it (Scheduler.scheduleOne,
    scheduler.go:431-484): Schedule with SCHEDULE_ONLY, then AssumePod of the pod with its nodeName
    set — on the resident kernel the Schedule commits tentatively and the matching AssumePod confirms
    it without a message; anything else in between undoes it."""

    def schedule_one(self, pod):
        from ksim.cache import FitError
        try:
            host = self.schedule(pod, assume=False)
        except FitError as e:
            return None, str(e)
        q = dict(pod, spec=dict(pod["spec"], nodeName=host))
        self.assume_pod(q)
        return host, None


class K8sCacheAdapterUndo(K8sCacheAdapter):
    """The adapter's pattern with a read of the device state between every other Schedule and its
    AssumePod: the read first undoes the tentative commit (an explicit UNDO message when the commit
    touched volume mounts or affinity counts, else the stop's exit message carries it), so the
    AssumePod commits again through the ordinary path — the same decisions and final state."""

    _k = 0

    def schedule_one(self, pod):
        from ksim.cache import FitError
        try:
            host = self.schedule(pod, assume=False)
        except FitError as e:
            return None, str(e)
        self._k += 1
        if self._k % 2:
            v = C.c_uint64()
            self._hcall("ksim_get_counter", C.byref(v))
        q = dict(pod, spec=dict(pod["spec"], nodeName=host))
        self.assume_pod(q)
        return host, None


IMPLS = {"py": SchedulerCache, "cpp": K8sCache, "adapter": K8sCacheAdapter, "adapter_undo": K8sCacheAdapterUndo}


@pytest.fixture(autouse=True, params=["one_wg", "scan"])
def per_pod_form(request, monkeypatch):
    """Every per-pod call in the single-workgroup kernel (clusters up to 8,192 nodes: every
    reduction in LDS) or in the multi-block scan kernel the larger clusters take: the same
    decisions either way."""
    monkeypatch.setenv("KSIM_ONE_WG", "0" if request.param == "scan" else "1")
    return request.param

POLICIES = {
    "default": scheduler.provider("DefaultProvider"),
    "talkintdata": scheduler.provider("TalkintDataProvider"),
    "lr_bra": (["GeneralPredicates", "CheckNodeCondition", "PodToleratesNodeTaints", "CheckNodeMemoryPressure",
                "CheckNodeDiskPressure"], [("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]),
    "no_priorities": (["GeneralPredicates", "CheckNodeCondition"], []),
}


def _drive(seed, policy, n_events, n_nodes, features=True, mode=abi.MODE_AUTO, impl="py", forget=0.0):
    preds, prios = POLICIES[policy]
    ref = R.SchedulerCache(set(preds), prios)
    dut = IMPLS[impl](preds, prios, device=0, mode=mode)
    decisions = 0
    try:
        for ev in event_stream(seed, ref, n_events, n_nodes, features, forget=forget):
            want = apply(ref, ev)
            got = apply(dut, ev)
            if ev[0] == "schedule":
                decisions += 1
                assert got == want, (ev[1]["metadata"]["name"], want, got)
        assert dut.last_node_index == ref.sched.last_node_index
        st = dut.node_state()
        assert dut.names == sorted(ref.listed, key=lambda s: s.encode())
        for i, name in enumerate(dut.names):
            ni = ref.nodes[name]
            got = (st["req_cpu"][i], st["req_mem"][i], st["nz_cpu"][i], st["nz_mem"][i], st["pod_count"][i],
                   st["port_count"][i])
            want = (ni.requested.cpu, ni.requested.mem, ni.nonzero_cpu, ni.nonzero_mem, len(ni.pods),
                    len(ni.used_ports))
            assert got == want, (name, want, got)
    finally:
        dut.close()
    return decisions


@pytest.mark.parametrize("impl", sorted(IMPLS))
@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("policy", sorted(POLICIES))
def test_event_stream_parity(seed, policy, impl):
    assert _drive(seed, policy, n_events=300, n_nodes=14, impl=impl) > 100


@pytest.mark.parametrize("impl", sorted(IMPLS))
@pytest.mark.parametrize("seed", range(3))
def test_event_stream_resource_only(seed, impl):
    """Resource-only pods (the fast kernels' pod shape) through the same event mix."""
    assert _drive(100 + seed, "lr_bra", n_events=400, n_nodes=20, features=False, impl=impl) > 150


@pytest.mark.parametrize("impl", sorted(IMPLS))
@pytest.mark.parametrize("seed", range(3))
def test_event_stream_with_forget(seed, impl):
    """ForgetPod of assumed pods whose binding failed (scheduler.go:412, cache.go:170-197) mixed into
    the stream: the pod's commit leaves the device row, every later decision matches."""
    assert _drive(200 + seed, "default", n_events=300, n_nodes=12, impl=impl, forget=0.08) > 80


@pytest.mark.parametrize("impl", sorted(IMPLS))
def test_cache_errors_match_reference_messages(impl):
    """cache.go's error paths, with its messages: assume of a cached pod, add of an added pod,
    update / remove of unknown or assumed pods, forget of a pod that was not assumed or was assumed
    elsewhere, remove of an unknown node."""
    preds, prios = POLICIES["lr_bra"]
    dut = IMPLS[impl](preds, prios, device=0)
    node = {"metadata": {"name": "n1"}, "status": {"allocatable": {"cpu": "4", "memory": "8Gi", "pods": "10"}}}
    pod = {"metadata": {"name": "p", "namespace": "ns", "uid": "u1"},
           "spec": {"nodeName": "n1", "containers": [{"resources": {"requests": {"cpu": "1"}}}]}}
    try:
        dut.add_node(node)
        dut.assume_pod(pod)
        with pytest.raises(KeyError, match="pod u1 is in the cache, so can't be assumed"):
            dut.assume_pod(pod)
        with pytest.raises(KeyError, match="pod u1 is not added to scheduler cache, so cannot be updated"):
            dut.update_pod(pod, pod)
        with pytest.raises(KeyError, match="pod u1 is not found in scheduler cache, so cannot be removed from it"):
            dut.remove_pod(pod)
        moved = {"metadata": pod["metadata"], "spec": dict(pod["spec"], nodeName="n2")}
        with pytest.raises(KeyError, match="pod u1 was assumed on n2 but assigned to n1"):
            dut.forget_pod(moved)
        dut.forget_pod(pod)
        assert int(dut.node_state()["req_cpu"][0]) == 0
        with pytest.raises(KeyError, match="pod u1 wasn't assumed so cannot be forgotten"):
            dut.forget_pod(pod)
        dut.add_pod(pod)
        with pytest.raises(KeyError, match="pod u1 was already in added state"):
            dut.add_pod(pod)
        with pytest.raises(KeyError, match="wasn't assumed so cannot be forgotten"):
            dut.forget_pod(pod)
        assert int(dut.node_state()["req_cpu"][0]) == 1000
        with pytest.raises(KeyError, match="node gone is not in the cache"):
            dut.remove_node({"metadata": {"name": "gone"}})
    finally:
        dut.close()


@pytest.mark.parametrize("impl", sorted(IMPLS))
def test_empty_cache_is_err_no_nodes(impl):
    preds, prios = POLICIES["default"]
    dut = IMPLS[impl](preds, prios, device=0)
    try:
        with pytest.raises(abi.NoNodesAvailable):
            dut.schedule({"metadata": {"name": "p"}, "spec": {"containers": [{}]}})
        dut.add_node({"metadata": {"name": "n"}, "status": {"allocatable": {"cpu": "1", "memory": "1Gi", "pods": "2"}}})
        assert dut.schedule({"metadata": {"name": "p"}, "spec": {"containers": [{}]}}) == "n"
        assert dut.last_node_index == 0  # a single fit does not call selectHost
    finally:
        dut.close()


@pytest.mark.parametrize("impl", sorted(IMPLS))
def test_schedule_only_leaves_cache_unchanged(impl):
    preds, prios = POLICIES["lr_bra"]
    dut = IMPLS[impl](preds, prios, device=0)
    try:
        for i in range(3):
            dut.add_node({"metadata": {"name": "n%d" % i},
                          "status": {"allocatable": {"cpu": "4", "memory": "8Gi", "pods": "10"}}})
        pod = {"metadata": {"name": "p"}, "spec": {"containers": [{"resources": {"requests": {"cpu": "1"}}}]}}
        hosts = [dut.schedule(pod) for _ in range(3)]
        assert hosts == ["n2", "n1", "n0"]  # ties rotate from the highest name; nothing committed
        assert int(dut.node_state()["req_cpu"].sum()) == 0
        assert dut.schedule(pod, assume=True) == "n2"
        assert list(dut.node_state()["req_cpu"]) == [0, 0, 1000]
    finally:
        dut.close()


def _volume_stream(seed, ref, n_events, n_nodes, claims):
    """event_stream with volumes on the scheduled and bound pods (namespace "ns")."""
    import random
    from events import event_stream
    from workloads import rnd_volume
    rng = random.Random(7000 + seed)
    for kind, x in event_stream(seed, ref, n_events, n_nodes, features=False):
        if kind in ("schedule", "add_pod") and "uid" not in x["metadata"] and x["metadata"].get("namespace") != "ns":
            x["metadata"]["namespace"] = "ns"
            if rng.random() < 0.6:
                x["spec"]["volumes"] = [rnd_volume(rng, claims) for _ in range(rng.randint(1, 3))]
        yield kind, x


@pytest.mark.parametrize("impl", sorted(IMPLS))
@pytest.mark.parametrize("seed", range(4))
def test_event_stream_with_volumes(seed, monkeypatch, impl):
    """Volume pods through the per-pod mirror: its volume tables are rebuilt from the cache's pods
    after node events and when new keys appear, and every decision matches the oracle's."""
    from workloads import volume_listers
    monkeypatch.setenv("KUBE_MAX_PD_VOLS", "3")
    pvs, pvcs, claims = volume_listers()
    preds = ["GeneralPredicates", "CheckNodeCondition", "NoDiskConflict", "MaxEBSVolumeCount",
             "MaxGCEPDVolumeCount", "MaxAzureDiskVolumeCount"]
    prios = [("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]
    custom = {k: v for k, v in R.volume_predicates(R.VolumeListers(pvs, pvcs), 3).items() if k in preds}
    ref = R.SchedulerCache(set(preds), prios, custom)
    dut = IMPLS[impl](preds, prios, device=0, pvs=pvs, pvcs=pvcs)
    decisions = fails = 0
    try:
        for ev in _volume_stream(seed, ref, 300, 10, claims):
            want = apply(ref, ev)
            got = apply(dut, ev)
            if ev[0] == "schedule":
                decisions += 1
                fails += want[0] is None
                assert got == want, (ev[1]["metadata"]["name"], want, got)
        assert dut.last_node_index == ref.sched.last_node_index
    finally:
        dut.close()
    assert decisions > 100


def _affinity_stream(seed, ref, n_events, n_nodes):
    """scheduleOne calls of pods with inter-pod (anti-)affinity terms and spread labels, pods bound
    elsewhere on listed nodes, confirmations, removals and node updates (no node removal: the
    reference errs on affinity pods cached under a node-less NodeInfo)."""
    import copy
    import random
    from workloads import rnd_affinity_nodes, rnd_affinity_pod
    rng = random.Random(9000 + seed)
    for node in rnd_affinity_nodes(rng, n_nodes):
        yield "add_node", node
    for k in range(n_events):
        names = list(ref.listed)
        added = sorted(key for key in ref.pod_states if key not in ref.assumed)
        assumed = sorted(ref.assumed)
        r = rng.random()
        if r < 0.6:
            yield "schedule", rnd_affinity_pod(rng, "p-%d" % k, p_aff=0.5)
        elif r < 0.7:
            p = rnd_affinity_pod(rng, "bound-%d" % k, p_aff=0.3)
            p["spec"]["nodeName"] = rng.choice(names)
            yield "add_pod", p
        elif r < 0.8 and assumed:
            yield "add_pod", copy.deepcopy(ref.pod_states[rng.choice(assumed)])
        elif r < 0.9 and added:
            yield "remove_pod", copy.deepcopy(ref.pod_states[rng.choice(added)])
        else:
            name = rng.choice(names)
            old = ref.nodes[name].node
            new = copy.deepcopy(old)
            lab = new["metadata"].get("labels") or {}
            lab["zone"] = "z%d" % rng.randint(0, 3)
            new["metadata"]["labels"] = lab
            yield "update_node", (old, new)


@pytest.mark.parametrize("impl", sorted(IMPLS))
@pytest.mark.parametrize("seed", range(4))
def test_event_stream_with_affinity_and_spread(seed, impl):
    """Inter-pod affinity and SelectorSpread pods through the per-pod mirror (incremental affinity
    index, tables reloaded only when it grows or after node events): every decision matches the
    oracle's cache."""
    from ksim.spread import SpreadListers
    svc = [{"metadata": {"namespace": ns}, "spec": {"selector": {"app": a}}} for ns, a in (("", "web"), ("ns1", "db"))]
    rss = [{"metadata": {"namespace": ""}, "spec": {"selector": {"matchLabels": {"tier": "fe"}}}}]
    preds, prios = POLICIES["default"]
    ref = R.SchedulerCache(set(preds), prios, spread=R.SpreadListers(services=svc, rss=rss))
    dut = IMPLS[impl](preds, prios, device=0, spread=SpreadListers(services=svc, rss=rss))
    decisions = 0
    try:
        for ev in _affinity_stream(seed, ref, 200, 12):
            want = apply(ref, ev)
            got = apply(dut, ev)
            if ev[0] == "schedule":
                decisions += 1
                assert got == want, (ev[1]["metadata"]["name"], want, got)
        assert dut.last_node_index == ref.sched.last_node_index
    finally:
        dut.close()
    assert decisions > 80


@pytest.mark.parametrize("impl", sorted(IMPLS))
def test_affinity_tables_load_only_on_growth(impl):
    """The per-pod path keeps the inter-pod affinity / SelectorSpread state incrementally
    (predicates/metadata.go:127-190): on a replicated workload — four pod templates, hostname
    anti-affinity on two of them, services selecting all — the tables load a handful of times while
    the index learns the templates, then never again over hundreds of Schedule + assume calls and
    removals; every decision still matches the oracle's cache."""
    import copy
    import random
    from ksim.spread import SpreadListers
    rng = random.Random(77)
    svc = [{"metadata": {"namespace": ""}, "spec": {"selector": {"app": a}}} for a in ("web", "db")]
    preds, prios = POLICIES["default"]
    ref = R.SchedulerCache(set(preds), prios, spread=R.SpreadListers(services=svc))
    dut = IMPLS[impl](preds, prios, device=0, spread=SpreadListers(services=svc))

    def template(k, name):
        app = ("web", "db", "web", "cache")[k]
        pod = {"metadata": {"name": name, "namespace": "", "uid": name, "labels": {"app": app, "tier": str(k)}},
               "spec": {"containers": [{"resources": {"requests": {"cpu": "100m", "memory": "64Mi"}}}]}}
        if k in (0, 1):
            pod["spec"]["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": {"matchLabels": {"app": app}}, "topologyKey": "kubernetes.io/hostname"}]}}
        return pod

    try:
        for i in range(40):
            node = {"metadata": {"name": "n-%02d" % i, "labels": {"kubernetes.io/hostname": "n-%02d" % i,
                                                                   "failure-domain.beta.kubernetes.io/zone": "z%d" % (i % 3)}},
                    "status": {"allocatable": {"cpu": "8", "memory": "16Gi", "pods": "110"}}}
            apply(ref, ("add_node", node))
            apply(dut, ("add_node", node))
        loads_after_warmup = None
        for k in range(400):
            if k == 40:
                loads_after_warmup = dut.aff_reloads
            added = sorted(key for key in ref.pod_states if key not in ref.assumed)
            if k % 10 == 9 and added:
                ev = ("remove_pod", copy.deepcopy(ref.pod_states[rng.choice(added)]))
            elif k % 10 == 8 and ref.assumed:
                ev = ("add_pod", copy.deepcopy(ref.pod_states[sorted(ref.assumed)[0]]))
            else:
                ev = ("schedule", template(rng.randrange(4), "p-%d" % k))
            want = apply(ref, ev)
            got = apply(dut, ev)
            if ev[0] == "schedule":
                assert got == want, (ev[1]["metadata"]["name"], want, got)
        assert dut.last_node_index == ref.sched.last_node_index
        assert dut.aff_reloads <= 8
        assert dut.aff_reloads == loads_after_warmup
    finally:
        dut.close()


@pytest.mark.parametrize("impl", sorted(IMPLS))
def test_volume_tables_grow_without_reload(impl):
    """Volume pods through the per-pod mirror: a pod that brings a new disk grows the device's
    volume tables (ksim_grow_volumes: keys, classes, refs, zone verdicts, more slots) while the
    device keeps every node's mounts, so the full reload happens once (no node events here) over
    hundreds of Schedule + assume calls and removals; every decision matches the oracle's cache."""
    import copy
    import random
    preds, prios = POLICIES["default"]
    ref = R.SchedulerCache(set(preds), prios)
    dut = IMPLS[impl](preds, prios, device=0)
    rng = random.Random(5)
    try:
        for i in range(24):
            node = {"metadata": {"name": "v-%02d" % i, "labels": {"kubernetes.io/hostname": "v-%02d" % i}},
                    "status": {"allocatable": {"cpu": "16", "memory": "32Gi", "pods": "110"}}}
            apply(ref, ("add_node", node))
            apply(dut, ("add_node", node))
        for k in range(360):
            added = sorted(key for key in ref.pod_states if key not in ref.assumed)
            if k % 9 == 8 and added:
                ev = ("remove_pod", copy.deepcopy(ref.pod_states[rng.choice(added)]))
            elif k % 9 == 7 and ref.assumed:
                ev = ("add_pod", copy.deepcopy(ref.pod_states[sorted(ref.assumed)[0]]))
            else:
                vols = []
                for v in range(rng.choice([1, 1, 2, 3])):
                    if rng.random() < 0.5:
                        vols.append({"name": "g%d" % v, "gcePersistentDisk": {"pdName": "pd-%d" % rng.randrange(150),
                                                                              "readOnly": rng.random() < 0.4}})
                    else:
                        vols.append({"name": "e%d" % v, "awsElasticBlockStore": {"volumeID": "vol-%d" % rng.randrange(150)}})
                name = "vp-%d" % k
                ev = ("schedule", {"metadata": {"name": name, "namespace": "", "uid": name},
                                   "spec": {"containers": [{"resources": {"requests": {"cpu": "100m"}}}], "volumes": vols}})
            want = apply(ref, ev)
            got = apply(dut, ev)
            if ev[0] == "schedule":
                assert got == want, (ev[1]["metadata"]["name"], want, got)
        assert dut.last_node_index == ref.sched.last_node_index
        assert dut.vol_loads == 1 and dut.vol_grows > 20
    finally:
        dut.close()


def _image_stream(seed, ref, n_events, n_nodes):
    """event_stream with status.images on the nodes (sizes across calculateScoreFromSize's buckets)
    and container images on the scheduled / bound pods."""
    import random
    from events import event_stream
    rng = random.Random(4000 + seed)
    catalog = [("reg/app:%d" % i, size) for i, size in enumerate([5, 30, 120, 400, 800, 1200])]

    def images(node):
        picks = rng.sample(catalog, rng.randint(0, 4))
        node.setdefault("status", {})["images"] = [{"names": [n, n + "@sha"], "sizeBytes": s * 1024 * 1024} for n, s in picks]

    for kind, x in event_stream(seed, ref, n_events, n_nodes, features=False):
        if kind == "add_node":
            images(x)
        elif kind == "update_node":
            images(x[1])
        elif kind in ("schedule", "add_pod") and "uid" not in x["metadata"]:
            for c in x["spec"]["containers"]:
                if rng.random() < 0.8:
                    c["image"] = rng.choice(catalog)[0]
        yield kind, x


@pytest.mark.parametrize("impl", sorted(IMPLS))
@pytest.mark.parametrize("seed", range(3))
def test_event_stream_with_image_locality(seed, impl):
    """ImageLocalityPriority (image_locality.go:39-88) weighted in the policy, nodes listing images
    that change on node updates: node images interned into label sets, pod images into classes, the
    bucketed score a per-(class, label set) addend; every decision matches the oracle's cache."""
    preds = ["GeneralPredicates", "CheckNodeCondition", "PodToleratesNodeTaints"]
    prios = [("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1), ("ImageLocalityPriority", 2)]
    ref = R.SchedulerCache(set(preds), prios)
    dut = IMPLS[impl](preds, prios, device=0)
    decisions = 0
    try:
        for ev in _image_stream(seed, ref, 250, 10):
            want = apply(ref, ev)
            got = apply(dut, ev)
            if ev[0] == "schedule":
                decisions += 1
                assert got == want, (ev[1]["metadata"]["name"], want, got)
        assert dut.last_node_index == ref.sched.last_node_index
    finally:
        dut.close()
    assert decisions > 80


@pytest.mark.parametrize("seed", range(2))
@pytest.mark.parametrize("name", ["absent_rank", "present_tier_disk", "service_affinity", "label_priorities"])
def test_event_stream_with_policy_arguments(seed, name):
    """A Policy's arguments through the C++ scheduler cache (ksim_k8s_cache_options.policy):
    CheckNodeLabelPresence on node rows as they are added / updated, CheckServiceAffinity's table
    and the label priorities' addends as label sets and classes are interned — decision by decision
    against the oracle's cache with the same Policy."""
    from ksim import policy
    from test_policy import GPU_POLICIES
    pol = policy.decode(GPU_POLICIES[name])
    preds, prios, lp = policy.key_sets(pol)
    sa = policy.service_affinity_labels(pol)
    args = policy.priority_arguments(pol)
    custom = {"CheckNodeLabelPresence": R.new_node_label_predicate(*lp)} if lp else {}
    if sa is not None:
        custom["CheckServiceAffinity"] = R.new_service_affinity_predicate(sa)
    cprios = {n: (R.node_label_priority(a[1], a[2]) if a[0] == "labelPreference" else R.service_anti_affinity_priority(a[1]))
              for n, a in args.items()}
    ref = R.SchedulerCache(set(preds), prios, custom)
    ref.sched = R.GenericScheduler(set(preds), list(prios), custom, custom_priorities=cprios)
    dut = K8sCache(preds, prios, label_presence=lp, service_affinity=sa, custom_priorities=args)
    decisions = 0
    try:
        for ev in event_stream(seed, ref, 300, 14, True):
            want = apply(ref, ev)
            got = apply(dut, ev)
            if ev[0] == "schedule":
                decisions += 1
                assert got == want, (ev[1]["metadata"]["name"], want, got)
        assert dut.last_node_index == ref.sched.last_node_index
    finally:
        dut.close()
    assert decisions > 100
