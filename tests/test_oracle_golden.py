"""Pins the CPU oracle (oracle/ksim_ref.py) against golden vectors transcribed from
the reference's own Go tests (tests/golden/make_golden.py)."""
import pytest

import ksim_ref as R
from golden_util import case_id, load


@pytest.mark.parametrize("c", load("quantity"), ids=case_id)
def test_quantity(c):
    assert R.q_milli(c["q"]) == c["milli"]
    assert R.q_value(c["q"]) == c["value"]


def _infos(nodes, pods):
    infos = [R.NodeInfo(n) for n in nodes]
    by = {ni.name: ni for ni in infos}
    for p in pods:
        nn = p["spec"].get("nodeName", "")
        if nn in by:
            by[nn].add_pod(p)
    return infos


@pytest.mark.parametrize("c", load("priorities"), ids=case_id)
def test_priority(c):
    infos = _infos(c["nodes"], c["pods"])
    scores = R.prioritize_nodes(c["pod"], infos, [(c["priority"], 1)])
    assert [[ni.name, s] for ni, s in zip(infos, scores)] == c["expect"]


@pytest.mark.parametrize("c", load("predicates"), ids=case_id)
def test_predicate(c):
    ni = R.NodeInfo(c["node"])
    for p in c["pods"]:
        ni.add_pod(p)
    ok, reasons = R.PREDICATES[c["predicate"]](c["pod"], ni)
    assert ok == c["fits"]
    if not ok and c["reasons"] is not None:
        assert reasons == c["reasons"]


def test_node_info_add_pod():
    (c,) = load("node_info")
    ni = R.NodeInfo(c["node"])
    for p in c["pods"]:
        ni.add_pod(p)
    e = c["expect"]
    assert (ni.requested.cpu, ni.requested.mem) == (e["requested_cpu"], e["requested_mem"])
    assert (ni.nonzero_cpu, ni.nonzero_mem) == (e["nonzero_cpu"], e["nonzero_mem"])
    assert len(ni.pods) == e["pod_count"]
    assert ni.used_ports == {tuple(x) for x in e["used_ports"]}


@pytest.mark.parametrize("c", load("prioritize"), ids=case_id)
def test_zero_request(c):
    infos = _infos(c["nodes"], c["pods"])
    scores = R.prioritize_nodes(c["pod"], infos, [tuple(x) for x in c["configs"]])
    if "expect_all_equal" in c:
        assert all(s == c["expect_all_equal"] for s in scores)
    else:
        assert all(s != c["expect_none_equal"] for s in scores)


@pytest.mark.parametrize("c", load("select_host"), ids=case_id)
def test_select_host(c):
    g = R.GenericScheduler([], [])
    got = [g.select_host([tuple(x) for x in c["list"]]) for _ in range(c["calls"])]
    assert set(got) <= set(c["possible"])
    # exact round-robin (derived, not pinned by the Go test): descending host-name order
    ties = sorted(c["possible"], key=lambda h: h.encode(), reverse=True)
    assert got == [ties[i % len(ties)] for i in range(c["calls"])]


def test_fit_error_message():
    (c,) = load("fit_error")
    msg = str(R.FitError(c["num_nodes"], c["failed"]))
    for s in c["contains"]:
        assert s in msg


@pytest.mark.parametrize("c", load("volumes"), ids=case_id)
def test_volume_predicate(c):
    """NoDiskConflict / MaxEBSVolumeCount / NoVolumeZoneConflict over the Go tests' fake PV / PVC
    listers (predicates_test.go:669-891, 1622-2039, 3694-3913)."""
    ni = R.NodeInfo(c["node"])
    for p in c["pods"]:
        ni.add_pod(p)
    preds = R.volume_predicates(R.VolumeListers(c["pvs"], c["pvcs"]), c["max_vols"])
    ok, reasons = preds[c["predicate"]](c["pod"], ni)
    assert ok == c["fits"]
    assert reasons == c["reasons"]


def test_get_max_vols():
    """TestGetMaxVols (predicates_test.go:4039-4083): the env value when it parses to a positive
    int, else the default."""
    assert R.get_max_vols(39, "") == 39
    assert R.get_max_vols(39, "2") == 2
    assert R.get_max_vols(39, "invalid") == 39
    assert R.get_max_vols(39, "-2") == 39
    assert R.get_max_vols(39, "0") == 39
    assert R.get_max_vols(39, "40") == 40


def test_volume_error_paths():
    """A PVC the simulator's (empty) listers cannot resolve: MaxPD counts it, VolumeZone errors on a
    zone-labelled node, VolumeBinding errors everywhere (predicates.go:376-383, 575-578, 1597-1600)."""
    p = {"metadata": {"name": "p", "namespace": "ns"}, "spec": {"volumes": [{"persistentVolumeClaim": {"claimName": "c"}}]}}
    plain = R.NodeInfo({"metadata": {"name": "a"}})
    zoned = R.NodeInfo({"metadata": {"name": "b", "labels": {R.ZONE_LABEL: "z1"}}})
    assert R.PREDICATES["MaxEBSVolumeCount"](p, plain) == (True, [])
    assert R.PREDICATES["NoVolumeZoneConflict"](p, plain) == (True, [])
    with pytest.raises(R.PredicateError):
        R.PREDICATES["NoVolumeZoneConflict"](p, zoned)
    with pytest.raises(R.PredicateError):
        R.PREDICATES["CheckVolumeBinding"](p, plain)
    noname = {"metadata": {}, "spec": {"volumes": [{"persistentVolumeClaim": {"claimName": ""}}]}}
    with pytest.raises(R.PredicateError):
        R.PREDICATES["MaxGCEPDVolumeCount"](noname, plain)


@pytest.mark.parametrize("c", load("spread"), ids=case_id)
def test_selector_spread(c):
    """SelectorSpreadPriority over services / RCs / RSs / StatefulSets (selector_spreading_test.go:43-812),
    every node listed (no predicates)."""
    infos = _infos(c["nodes"], c["pods"])
    listers = R.SpreadListers(c["services"], c["rcs"], c["rss"], c["sss"])
    scores = R.prioritize_nodes(c["pod"], infos, [("SelectorSpreadPriority", 1)], spread=listers)
    assert {ni.name: s for ni, s in zip(infos, scores)} == c["expect"]


@pytest.mark.parametrize("c", load("label_priorities"), ids=case_id)
def test_label_priorities(c):
    """Policy priorities with arguments: labelPreference (node_label_test.go:30-128) and
    serviceAntiAffinity (TestZoneSpreadPriority, selector_spreading_test.go:605-760)."""
    infos = _infos(c["nodes"], c["pods"])
    if c["kind"] == "labelPreference":
        custom = {"P": R.node_label_priority(c["label"], c["presence"])}
    else:
        custom = {"P": R.service_anti_affinity_priority(c["label"], R.SpreadListers(c["services"]))}
    scores = R.prioritize_nodes(c["pod"], infos, [("P", 1)], custom=custom)
    assert {ni.name: s for ni, s in zip(infos, scores)} == c["expect"]


@pytest.mark.parametrize("c", load("service_affinity"), ids=case_id)
def test_service_affinity(c):
    """CheckServiceAffinity (TestServiceAffinity, predicates_test.go:1460-1620)."""
    ni = R.NodeInfo(c["node"])
    pred = R.new_service_affinity_predicate(c["labels"], c["services"], c["pods"], c["nodes"])
    ok, reasons = pred(c["pod"], ni)
    assert ok == c["fits"]
    assert reasons == ([] if ok else [R.R_SERVICE_AFFINITY])
