"""SelectorSpread through the affinity tables (ksim/affinity.py + ksim/spread.py): every pod's spread
counted pair holds, per node, the oracle's CalculateSpreadPriorityMap count (selector_spreading.go:66-114)
— on the reference's golden cases and on random clusters — and the zone pseudo key groups the nodes
as utilnode.GetZoneKey does."""
import pytest

import ksim_ref as R
from golden_util import case_id, load
from ksim import affinity, ingest, spread
from workloads import rnd_spread_workload


def _counts(cl, k):
    t = cl.affinity
    a = int(cl.pods["aff_class"][k])
    if a == 0:
        return None
    c = int(t["spread_pair"][a - 1])
    if c < 0:
        return None
    off = int(t["pair_off"][c])
    return [int(x) for x in t["cnt"][off:off + cl.n_nodes]]


@pytest.mark.parametrize("c", load("spread"), ids=case_id)
def test_golden_spread_counts(c):
    lst = spread.SpreadListers(c["services"], c["rcs"], c["rss"], c["sss"])
    cl = ingest.Cluster.from_objects(c["nodes"], c["pods"], [c["pod"]], spread=lst)
    infos = [R.NodeInfo(x) for x in sorted(c["nodes"], key=lambda x: x["metadata"]["name"].encode())]
    by = {ni.name: ni for ni in infos}
    for p in c["pods"]:
        if p["spec"].get("nodeName") in by:
            by[p["spec"]["nodeName"]].add_pod(p)
    sels = R.SpreadListers(c["services"], c["rcs"], c["rss"], c["sss"]).selectors(c["pod"])
    want = [R.selector_spread_map(c["pod"], ni, sels) for ni in infos]
    got = _counts(cl, 0)
    assert (got is None) == (not sels)
    if got is not None:
        assert got == want


@pytest.mark.parametrize("services_only", [False, True])
@pytest.mark.parametrize("seed", range(6))
def test_random_spread_counts_and_zones(seed, services_only):
    nodes, running, pods, objs = rnd_spread_workload(seed)
    lst = spread.SpreadListers(**objs)
    cl = ingest.Cluster.from_objects(nodes, running, pods, spread=lst, spread_services_only=services_only)
    oracle = R.SpreadListers(**objs)
    infos = [R.NodeInfo(x) for x in sorted(nodes, key=lambda x: x["metadata"]["name"].encode())]
    by = {ni.name: ni for ni in infos}
    for p in running:
        by[p["spec"]["nodeName"]].add_pod(p)
    seen = 0
    for k, p in enumerate(pods):
        sels = oracle.selectors(p, services_only)
        got = _counts(cl, k)
        assert (got is None) == (not sels), k
        if got is not None:
            assert got == [R.selector_spread_map(p, ni, sels) for ni in infos]
            seen += 1
    assert seen > 10
    t = cl.affinity
    zk = int(t["zone_key"])
    assert zk >= 0
    zones = [R.zone_key(ni.node) for ni in infos]
    dom = [int(x) for x in t["dom"][zk]]
    for i in range(len(infos)):
        assert (dom[i] < 0) == (zones[i] == "")
        for j in range(len(infos)):
            if dom[i] >= 0 and dom[j] >= 0:
                assert (dom[i] == dom[j]) == (zones[i] == zones[j])
