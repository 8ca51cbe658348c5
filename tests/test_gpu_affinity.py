"""Inter-pod affinity on the GPU (MatchInterPodAffinity + InterPodAffinityPriority through
ksim_load_affinity and the launch-mode kernels) against the object-level oracle
(ksim_ref.interpod_affinity_matches / interpod_affinity_priority, pinned by the reference's own
test tables in test_oracle_interpod.py): whole simulations with every placement, FitError text and
the final lastNodeIndex identical; the per-pod entry points (ksim_schedule_one, ksim_pod_add /
remove) keeping the counts consistent with the batch path."""
import ctypes as C

import numpy as np
import pytest

import ksim_ref as R
from ksim import abi, ingest, scheduler
from workloads import rnd_affinity_workload

pytestmark = pytest.mark.gpu

POLICIES = {
    "default": scheduler.provider("DefaultProvider"),
    "talkintdata": scheduler.provider("TalkintDataProvider"),
    "ipa_heavy": (list(scheduler.DEFAULT_PREDICATES), [("InterPodAffinityPriority", 7), ("LeastRequestedPriority", 1),
                                                         ("TaintTolerationPriority", 2)]),
    "ipa_only": (["MatchInterPodAffinity", "PodFitsResources"], [("InterPodAffinityPriority", 1)]),
    "predicate_only": (["MatchInterPodAffinity", "GeneralPredicates"], [("MostRequestedPriority", 1)]),
}
MODES = [abi.MODE_LAUNCH, abi.MODE_AUTO, abi.MODE_TREE, abi.MODE_PERSISTENT]


def _check(nodes, running, pods, preds, prios, mode, hard_weight=10):
    want, want_lni = R.simulate(nodes, running, pods, set(preds), list(prios)) if hard_weight == 10 else (None, None)
    if want is None:
        raise AssertionError("hard weight")
    cc = scheduler.ClusterCapacity(nodes, running, pods, predicates=preds, priorities=prios, mode=mode)
    rep = cc.run()
    got = {n: (h, None) for n, h in rep.successful}
    got.update({n: (None, m) for n, m in rep.failed})
    assert [n for n, _ in rep.successful] == [n for n, h, _ in want if h is not None]
    for name, host, msg in want:
        assert got[name] == (host, msg), name
    assert rep.last_node_index == want_lni
    return want


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("policy", sorted(POLICIES))
@pytest.mark.parametrize("seed", range(3))
def test_affinity_simulation_matches_oracle(seed, policy, mode):
    preds, prios = POLICIES[policy]
    nodes, running, pods = rnd_affinity_workload(seed, n_nodes=18 + 7 * seed, n_pods=90, n_running=12)
    want = _check(nodes, running, pods, preds, prios, mode)
    if "MatchInterPodAffinity" in preds:
        assert any(m and "affinity" in m for _, _, m in want)   # the predicate decided something


@pytest.mark.parametrize("policy", sorted(POLICIES))
@pytest.mark.parametrize("seed", range(3))
def test_affinity_two_launch_form_matches_oracle(seed, policy, monkeypatch):
    """Launch form with pass A as its own launch (KSIM_FUSE_A=0) instead of fused into the scan."""
    monkeypatch.setenv("KSIM_FUSE_A", "0")
    preds, prios = POLICIES[policy]
    nodes, running, pods = rnd_affinity_workload(seed, n_nodes=18 + 7 * seed, n_pods=90, n_running=12)
    _check(nodes, running, pods, preds, prios, abi.MODE_LAUNCH)


@pytest.mark.parametrize("policy", ["default", "ipa_heavy"])
def test_fused_barrier_timeout_recovers(policy, monkeypatch):
    """The fused pass-A grid barrier bailing out (KSIM_BARRIER_TICKS=0: every block that has to wait
    gives up at once, as when the grid is not co-resident after all): the launch at the cursor
    commits nothing, the rest of the graph exits at its entry check, and the runtime re-arms the
    tickets and finishes with pass A as its own launch — placements still identical to the oracle."""
    monkeypatch.setenv("KSIM_BARRIER_TICKS", "0")
    preds, prios = POLICIES[policy]
    nodes, running, pods = rnd_affinity_workload(4, n_nodes=600, n_pods=60, n_running=12, p_aff=0.6)
    _check(nodes, running, pods, preds, prios, abi.MODE_LAUNCH)


@pytest.mark.parametrize("seed", range(3))
def test_mixed_affinity_and_resource_only_pods(seed):
    """Mostly term-free pods (tree / fast kernels) interleaved with affinity pods (launch kernels):
    the counts the launch kernels read must include every placed pod whose labels some term
    selects, whatever path placed it."""
    nodes, running, pods = rnd_affinity_workload(50 + seed, n_nodes=30, n_pods=160, n_running=8, p_aff=0.15)
    for mode in (abi.MODE_TREE, abi.MODE_AUTO):
        _check(nodes, running, pods, *POLICIES["default"], mode=mode)


def test_larger_cluster_many_terms():
    nodes, running, pods = rnd_affinity_workload(7, n_nodes=300, n_pods=220, n_running=60, p_aff=0.8)
    _check(nodes, running, pods, *POLICIES["ipa_heavy"], mode=abi.MODE_AUTO)


def test_hostname_self_affinity_and_spread():
    """Typical deployment shapes: a required self-anti-affinity per hostname (one replica per node)
    and a required zone affinity to a service."""
    nodes = [{"metadata": {"name": "n%d" % i, "labels": {"kubernetes.io/hostname": "n%d" % i, "zone": "z%d" % (i % 3)}},
              "status": {"allocatable": {"cpu": "8", "memory": "16Gi", "pods": "110"}}} for i in range(9)]
    anti = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"app": "web"}}, "topologyKey": "kubernetes.io/hostname"}]}}
    aff = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"app": "db"}}, "topologyKey": "zone"}]}}
    running = [{"metadata": {"name": "db0", "uid": "db0", "labels": {"app": "db"}}, "spec": {"nodeName": "n4", "containers": [{}]}}]
    pods = [{"metadata": {"name": "web%d" % k, "labels": {"app": "web"}}, "spec": {"containers": [{}], "affinity": anti}}
            for k in range(12)]
    pods += [{"metadata": {"name": "api%d" % k, "labels": {"app": "api"}}, "spec": {"containers": [{}], "affinity": aff}}
             for k in range(5)]
    for mode in (abi.MODE_LAUNCH, abi.MODE_AUTO):
        want = _check(nodes, running, pods, *POLICIES["default"], mode=mode)
    placed_web = [h for n, h, _ in want if n.startswith("web") and h]
    assert len(placed_web) == 9 and len(set(placed_web)) == 9
    assert {h for n, h, _ in want if n.startswith("api")} <= {"n1", "n4", "n7"}


def _handle_for(cl, preds, prios):
    return scheduler.GenericScheduler(cl, preds, prios, device=0, mode=abi.MODE_LAUNCH)


def test_schedule_one_matches_batch():
    """ksim_schedule_one (+ assume) pod by pod on one handle == ksim_schedule on another."""
    preds, prios = POLICIES["default"]
    nodes, running, pods = rnd_affinity_workload(21, n_nodes=25, n_pods=60)
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order)
    batch = _handle_for(cl, preds, prios)
    one = _handle_for(cl, preds, prios)
    try:
        out, reasons, _ = batch.schedule()
        for k in range(len(order)):
            pod = abi.Pod.from_buffer_copy(cl.pods[k].tobytes())
            ports = cl.pod_ports
            sc = cl.pod_scalars
            res = abi.Result()
            one.h.call("ksim_schedule_one", C.byref(pod), abi.vptr(ports), len(ports), abi.vptr(sc), len(sc),
                       abi.SCHEDULE_ASSUME, C.byref(res))
            assert res.node == out[k], k
            if res.node < 0:
                assert list(res.reasons) == list(reasons[k]), k
        assert one.last_node_index == batch.last_node_index
    finally:
        batch.close()
        one.close()


def test_pod_remove_and_add_restore_counts():
    """ksim_pod_remove then ksim_pod_add of placed affinity pods leaves every later decision as
    if nothing happened (the counts return to the same values)."""
    preds, prios = POLICIES["ipa_heavy"]
    nodes, running, pods = rnd_affinity_workload(33, n_nodes=20, n_pods=70)
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order)
    a = _handle_for(cl, preds, prios)
    b = _handle_for(cl, preds, prios)
    try:
        half = len(order) // 2
        out_a, _, _ = a.schedule(0, half)
        out_b, _, _ = b.schedule(0, half)
        assert np.array_equal(out_a, out_b)
        ports, sc = cl.pod_ports, cl.pod_scalars
        for k in range(half):
            if out_b[k] < 0:
                continue
            pod = abi.Pod.from_buffer_copy(cl.pods[k].tobytes())
            b.h.call("ksim_pod_remove", int(out_b[k]), C.byref(pod), abi.vptr(ports), len(ports), abi.vptr(sc), len(sc))
        for k in range(half):
            if out_b[k] < 0:
                continue
            pod = abi.Pod.from_buffer_copy(cl.pods[k].tobytes())
            b.h.call("ksim_pod_add", int(out_b[k]), C.byref(pod), abi.vptr(ports), len(ports), abi.vptr(sc), len(sc))
        rest_a, _, _ = a.schedule(half)
        rest_b, _, _ = b.schedule(half)
        assert np.array_equal(rest_a, rest_b)
    finally:
        a.close()
        b.close()


def test_node_event_makes_tables_stale():
    preds, prios = POLICIES["default"]
    nodes, running, pods = rnd_affinity_workload(5, n_nodes=8, n_pods=10)
    cl = ingest.Cluster.from_objects(nodes, running, pods)
    g = _handle_for(cl, preds, prios)
    try:
        g.h.call("ksim_node_remove", 0)
        with pytest.raises(abi.KsimError) as ei:
            g.schedule()
        assert ei.value.code == abi.E_STATE
    finally:
        g.close()


def test_malformed_tables_are_rejected():
    preds, prios = POLICIES["default"]
    nodes, running, pods = rnd_affinity_workload(6, n_nodes=8, n_pods=10)
    cl = ingest.Cluster.from_objects(nodes, running, pods)
    g = _handle_for(cl, preds, prios)
    from ksim.affinity import tables_struct
    try:
        for field, bad in (("dom", lambda d: d.__setitem__((2, 0), 10 ** 6)),
                           ("pair_off", lambda d: d.__setitem__(0, 10 ** 9)),
                           ("carry_key", lambda d: d.__setitem__(0, 99))):
            T = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in cl.affinity.items()}
            if T[field].size == 0 or (field == "carry_key" and T["n_carry"] == 0):
                continue
            bad(T[field])
            with pytest.raises(abi.KsimError) as ei:
                g.h.call("ksim_load_affinity", C.byref(tables_struct(T)))
            assert ei.value.code == abi.E_INVAL, field
    finally:
        g.close()
