"""The oracle's inter-pod affinity restatement against the reference's own test tables:
TestInterPodAffinity / TestInterPodAffinityWithMultipleNodes (predicates_test.go:2168-3146) and
TestInterPodAffinityPriority / TestHardPodAffinitySymmetricWeight (interpod_affinity_test.go:
42-615), read into tests/golden/interpod_*.json by tests/golden/make_golden.py.  Each case is
evaluated under its Go harness's semantics (see make_golden.py).  CPU only."""
import pytest

import ksim_ref as R
from golden_util import case_id, load


def _name(o):
    return (o.get("metadata") or {}).get("name", "")


def _node_name(p):
    return (p.get("spec") or {}).get("nodeName", "")


@pytest.mark.parametrize("c", load("interpod_predicates"), ids=case_id)
def test_interpod_predicate_golden(c):
    nodes = c["nodes"]
    by_name = {_name(n): n for n in nodes}
    for node in nodes:
        on_node = [p for p in c["pods"] if _node_name(p) == _name(node)]
        if c["single_node"]:      # FakeNodeInfo: every pod's node is the test node
            all_pods = [(p, node) for p in c["pods"]]
        else:                     # FakeNodeListInfo: pods resolve to their own node
            all_pods = [(p, by_name[_node_name(p)]) for p in c["pods"]]
        node_pods = [(p, node) for p in on_node]
        meta = R.matching_anti_affinity_terms(c["pod"], all_pods if c["nometa"] else node_pods)
        fits, reasons, _ = R.interpod_affinity_matches(c["pod"], node, meta, all_pods, node_pods)
        if not fits:
            assert reasons == c["reasons"][_name(node)], _name(node)
        if (R._affinity(c["pod"]).get("nodeAffinity") is not None) and not c["single_node"]:
            fits = fits and R.pod_matches_node_labels(c["pod"], node)   # the multi-node harness ANDs it
        assert fits == c["fits"][_name(node)], _name(node)


@pytest.mark.parametrize("c", load("interpod_priorities"), ids=case_id)
def test_interpod_priority_golden(c):
    infos = {}
    for n in c["nodes"]:
        infos[_name(n)] = R.NodeInfo(n)
    for p in c["pods"]:            # CreateNodeNameToInfoMap: pods of unknown nodes get a node-less info
        infos.setdefault(_node_name(p), R.NodeInfo()).add_pod(p)
    got = R.interpod_affinity_priority(c["pod"], list(infos.values()), c["nodes"], c["hard_weight"])
    assert {_name(n): s for n, s in zip(c["nodes"], got)} == c["expect"]


def test_selector_semantics():
    assert R.label_selector_as_selector(None) is R.NOTHING
    assert R.label_selector_as_selector({}) == []
    with pytest.raises(R.AffinityError):
        R.label_selector_as_selector({"matchExpressions": [{"key": "a", "operator": "Gt", "values": ["1"]}]})
    with pytest.raises(R.AffinityError):
        R.label_selector_as_selector({"matchExpressions": [{"key": "a", "operator": "In"}]})
    p = {"metadata": {"namespace": "ns", "labels": {"a": "1"}}}
    assert R.pod_matches_term(p, {"ns"}, [])
    assert not R.pod_matches_term(p, {"other"}, [])
    assert not R.pod_matches_term(p, {"ns"}, R.NOTHING)
    a = {"metadata": {"labels": {"zone": "z"}}}
    assert R.same_topology(a, {"metadata": {"labels": {"zone": "z"}}}, "zone")
    assert not R.same_topology(a, {"metadata": {}}, "zone")
    assert not R.same_topology(a, a, "")
