"""GPU parity of SelectorSpreadPriority / ServiceSpreadingPriority with services, RCs, RSs and
StatefulSets (selector_spreading.go:66-174): the reference's golden cases through the kernels'
pass-A reductions (maxCountByNodeName, countsByZone) and the scan's float64 reduce — checked by
where selectHost puts the pod for every lastNodeIndex over two periods — and random simulations
against the object oracle (placements, FitError texts, lastNodeIndex)."""
import pytest

import ksim_ref as R
from golden_util import case_id, load
from ksim import abi, ingest, scheduler, spread
from workloads import rnd_spread_workload

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("c", load("spread"), ids=case_id)
def test_golden_spread_selects_on_gpu(c):
    expect = c["expect"]
    best = max(expect.values())
    tied = sorted((h for h, s in expect.items() if s == best), key=lambda h: h.encode(), reverse=True)
    lst = spread.SpreadListers(c["services"], c["rcs"], c["rss"], c["sss"])
    for k in range(2 * len(tied)):
        cl = ingest.Cluster.from_objects(c["nodes"], c["pods"], [c["pod"]], spread=lst)
        g = scheduler.GenericScheduler(cl, [], [("SelectorSpreadPriority", 1)], mode=abi.MODE_AUTO, last_node_index=k)
        out, _, _ = g.schedule(0, 1)
        assert cl.names[int(out[0])] == tied[k % len(tied)], (k, tied)
        g.close()


POLICIES = {
    "default": scheduler.provider("DefaultProvider"),
    "service_spreading": (["GeneralPredicates"], [("ServiceSpreadingPriority", 2), ("LeastRequestedPriority", 1)]),
    "spread_heavy": (["GeneralPredicates", "PodToleratesNodeTaints"],
                     [("SelectorSpreadPriority", 5), ("BalancedResourceAllocation", 1)]),
}


@pytest.mark.parametrize("fuse", ["fused", "two_launch"])
@pytest.mark.parametrize("policy", sorted(POLICIES))
@pytest.mark.parametrize("seed", range(4))
def test_spread_simulation_matches_oracle(seed, policy, fuse, monkeypatch):
    """Both launch forms: pass A fused into the scan (grid barrier) and as its own launch."""
    if fuse == "two_launch":
        monkeypatch.setenv("KSIM_FUSE_A", "0")
    nodes, running, pods, objs = rnd_spread_workload(seed, zones=seed != 3)
    preds, prios = POLICIES[policy]
    want, want_lni = R.simulate(nodes, running, pods, set(preds), list(prios), spread=R.SpreadListers(**objs))
    cc = scheduler.ClusterCapacity(nodes, running, pods, predicates=preds, priorities=prios,
                                   spread=spread.SpreadListers(**objs))
    assert cc.cluster.spread_active
    rep = cc.run()
    got = {name: (host, None) for name, host in rep.successful}
    got.update({name: (None, msg) for name, msg in rep.failed})
    assert [n for n, _ in rep.successful] == [n for n, h, _ in want if h is not None]
    for name, host, msg in want:
        assert got[name] == (host, msg), name
    assert rep.last_node_index == want_lni


def test_schedule_one_with_spread_matches_batch():
    """ksim_schedule_one (+ assume) pod by pod == ksim_schedule: pass A and the zone sums run for
    the single-pod launch as well (the accumulators are zeroed by each pass)."""
    import ctypes as C
    nodes, running, pods, objs = rnd_spread_workload(1, n_pods=50)
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order, spread=spread.SpreadListers(**objs))
    preds, prios = POLICIES["default"]
    batch = scheduler.GenericScheduler(cl, preds, prios, mode=abi.MODE_LAUNCH)
    one = scheduler.GenericScheduler(cl, preds, prios, mode=abi.MODE_LAUNCH)
    try:
        out, reasons, _ = batch.schedule()
        for k in range(len(order)):
            pod = abi.Pod.from_buffer_copy(cl.pods[k].tobytes())
            res = abi.Result()
            one.h.call("ksim_schedule_one", C.byref(pod), abi.vptr(cl.pod_ports), len(cl.pod_ports),
                       abi.vptr(cl.pod_scalars), len(cl.pod_scalars), abi.SCHEDULE_ASSUME, C.byref(res))
            assert res.node == out[k], k
        assert one.last_node_index == batch.last_node_index
    finally:
        batch.close()
        one.close()
