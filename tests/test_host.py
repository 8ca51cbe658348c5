"""CPU-only tests of the host side: library exports, quantity/selector semantics, ingest
tables and policy mapping (no compute calls — there is no GPU here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from golden_util import case_id, load
from ksim import abi, ingest, labels, quantity, scheduler

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "ksim.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(ksim_\w+)\(", src, re.M)))


def test_library_exports_every_header_symbol():
    L = abi.lib()
    fns = header_functions()
    assert len(fns) >= 12
    for f in fns:
        assert hasattr(L, f), f
    assert sorted(fns) == sorted(abi.EXPORTS)
    assert L.ksim_abi_version() == abi.ABI_VERSION == 7


def test_create_without_device_fails_loudly():
    cfg = scheduler.make_config(["GeneralPredicates"], [("LeastRequestedPriority", 1)])
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(abi.KsimError):
        abi.Handle(cfg)


@pytest.mark.parametrize("c", load("quantity"), ids=case_id)
def test_quantity_golden(c):
    assert quantity.milli_value(c["q"]) == c["milli"]
    assert quantity.value(c["q"]) == c["value"]


@pytest.mark.parametrize("c", [c for c in load("predicates") if c["predicate"] == "MatchNodeSelector"], ids=case_id)
def test_selector_golden(c):
    lab = c["node"]["metadata"].get("labels") or {}
    assert labels.pod_matches_node_labels(c["pod"]["spec"], lab) == c["fits"]


def _cluster_for(c):
    node = c["node"]
    pods = c.get("pods", [])
    return ingest.Cluster.from_objects([node], pods, [c["pod"]])


@pytest.mark.parametrize("c", [c for c in load("predicates") if c["predicate"] == "PodToleratesNodeTaints"], ids=case_id)
def test_taint_tables_golden(c):
    cl = _cluster_for(c)
    t = cl.tables
    ts = int(cl.cols["taint_set"][0])
    ok = bool((t["taint_ok"][0, ts >> 5] >> (ts & 31)) & 1)
    assert ok == c["fits"]


@pytest.mark.parametrize("c", [c for c in load("predicates") if c["predicate"] == "PodFitsResources"], ids=case_id)
def test_resource_ingest(c):
    """The pod descriptor carries GetResourceRequest; the node row carries
    allocatable + AddPod sums: check the predicate arithmetic on the host copy."""
    cl = _cluster_for(c)
    p = cl.pods[0]
    col = cl.cols
    fails = []
    if col["pod_count"][0] + 1 > col["allowed_pods"][0]:
        fails.append("Insufficient pods")
    if p["flags"] & abi.POD_ANY_REQUEST:
        if col["alloc_cpu"][0] < p["req_cpu"] + col["req_cpu"][0]:
            fails.append("Insufficient cpu")
        if col["alloc_mem"][0] < p["req_mem"] + col["req_mem"][0]:
            fails.append("Insufficient memory")
        if col["alloc_eph"][0] < p["req_eph"] + col["req_eph"][0]:
            fails.append("Insufficient ephemeral-storage")
        for s in cl.pod_scalars[p["scalar_off"]:p["scalar_off"] + p["scalar_cnt"]]:
            k = int(s["col"])
            if col["alloc_scalar"][k, 0] < s["req"] + col["req_scalar"][k, 0]:
                fails.append("Insufficient " + cl.scalar_names.items[k])
    assert (not fails) == c["fits"]
    if not c["fits"]:
        assert sorted(fails) == sorted(c["reasons"])


def test_node_info_add_pod_ingest():
    (c,) = load("node_info")
    cl = ingest.Cluster.from_objects([c["node"]], c["pods"], [])
    e = c["expect"]
    col = cl.cols
    assert (col["req_cpu"][0], col["req_mem"][0]) == (e["requested_cpu"], e["requested_mem"])
    assert (col["nz_cpu"][0], col["nz_mem"][0]) == (e["nonzero_cpu"], e["nonzero_mem"])
    assert col["pod_count"][0] == e["pod_count"]
    keys = {int(k) for k in col["ports"][:col["port_count"][0], 0]}
    want = {ingest.abi_port_key(cl.ips.ids[ip], cl.protos.ids[pr], port) for ip, pr, port in e["used_ports"]}
    assert keys == want


def test_nodes_sorted_bytewise():
    names = ["test-999.test.com", "test-1474.test.com", "B", "a", "test-10.test.com"]
    nodes = [{"metadata": {"name": n}, "status": {"allocatable": {"cpu": "1", "memory": "1", "pods": "1"}}} for n in names]
    cl = ingest.Cluster.from_objects(nodes, [], [])
    assert cl.names == sorted(names, key=lambda s: s.encode())
    assert cl.names[0] == "B"


def test_policy_mapping():
    p, q = scheduler.provider("TalkintDataProvider")
    cfg = scheduler.make_config(p, q)
    assert cfg.weights[abi.W_MOST] == 1 and cfg.weights[abi.W_LEAST] == 0
    assert cfg.const_score == 10 + 0 + 10 * 10000
    assert cfg.predicates & abi.P_GENERAL and cfg.predicates & abi.P_CHECK_NODE_CONDITION
    with pytest.raises(abi.KsimUnsupported):
        scheduler.make_config(["NoSuchPredicate"], [])
    with pytest.raises(abi.KsimUnsupported):
        scheduler.make_config([], [("NoSuchPriority", 1)])
    assert scheduler.make_config([], [("ImageLocalityPriority", 1)]).const_score == 0   # no node images
    assert scheduler.make_config([], []).no_priorities == 1


def test_unsupported_pods_rejected():
    n = [{"metadata": {"name": "n"}, "status": {"allocatable": {"cpu": "1", "pods": "10"}}}]
    # inter-pod affinity inputs on which the reference errors instead of placing
    term = {"labelSelector": {"matchLabels": {"a": "b"}}}
    p = {"metadata": {"name": "p"}, "spec": {"affinity": {"podAntiAffinity": {
        "requiredDuringSchedulingIgnoredDuringExecution": [term]}}}}                 # no topologyKey
    with pytest.raises(abi.KsimUnsupported):
        ingest.Cluster.from_objects(n, [], [p])
    bad = {"labelSelector": {"matchExpressions": [{"key": "a", "operator": "Gt", "values": ["1"]}]}, "topologyKey": "z"}
    p = {"metadata": {"name": "p"}, "spec": {"affinity": {"podAffinity": {
        "requiredDuringSchedulingIgnoredDuringExecution": [bad]}}}}                  # not a pod selector operator
    with pytest.raises(abi.KsimUnsupported):
        ingest.Cluster.from_objects(n, [], [p])
    ok = dict(term, topologyKey="zone")
    p = {"metadata": {"name": "p"}, "spec": {"affinity": {"podAffinity": {
        "requiredDuringSchedulingIgnoredDuringExecution": [ok]}}}}
    assert ingest.Cluster.from_objects(n, [], [p]).affinity is not None
    r = {"metadata": {"name": "r"}, "spec": {"nodeName": "gone"}}                      # bound to an unknown node
    with pytest.raises(abi.KsimUnsupported):
        ingest.Cluster.from_objects(n, [r], [p])
    # a PVC the simulator's empty listers cannot resolve: MaxPD counts it, but CheckVolumeBinding
    # errs (scheduler_binder.go:290-320) and so does VolumeZone on a zone-labelled node
    p = {"metadata": {"name": "p"}, "spec": {"volumes": [{"persistentVolumeClaim": {"claimName": "c"}}]}}
    cl = ingest.Cluster.from_objects(n, [], [p])
    assert cl.pods["vol_class"][0] == 1
    with pytest.raises(abi.KsimUnsupported):
        scheduler.check_volume_support(cl, scheduler.provider("DefaultProvider")[0])
    scheduler.check_volume_support(cl, ["NoDiskConflict", "MaxEBSVolumeCount", "NoVolumeZoneConflict"])
    zn = [dict(n[0], metadata={"name": "n", "labels": {"failure-domain.beta.kubernetes.io/zone": "z"}})]
    with pytest.raises(abi.KsimUnsupported):
        scheduler.check_volume_support(ingest.Cluster.from_objects(zn, [], [p]), ["NoVolumeZoneConflict"])
    two = {"metadata": {"name": "p"}, "spec": {"volumes": [{"rbd": {}, "iscsi": {}}]}}
    with pytest.raises(abi.KsimUnsupported):
        ingest.Cluster.from_objects(n, [], [two])


def test_fit_error_message_format():
    (c,) = load("fit_error")
    hist = np.zeros(abi.NREASONS, np.int32)
    hist[abi.R_MEM_PRESSURE] = 1
    hist[abi.R_DISK_PRESSURE] = 2
    msg = scheduler.fit_error_message(c["num_nodes"], hist)
    for s in c["contains"]:
        assert s in msg
    assert msg == "0/3 nodes are available: 1 node(s) had memory pressure, 2 node(s) had disk pressure."


def test_image_locality_addends_match_goldens():
    """ImageLocalityPriority (image_locality.go:39-88) with node images: node image sizes are
    interned into the label sets, the pod's container images into its class, and the per-(class,
    label set) score becomes a NodeAffinity-class addend (scheduler.class_tables_for).  On the
    reference's TestImageLocalityPriority cases the addend of each node's class is the golden score;
    a cluster built without image interning refuses the priority."""
    import json
    import os
    from ksim import ingest, scheduler
    cases = [c for c in json.load(open(os.path.join(os.path.dirname(__file__), "golden", "priorities.json")))
             if c["priority"] == "ImageLocalityPriority"]
    assert len(cases) == 3
    for c in cases:
        cl = ingest.Cluster.from_objects(c["nodes"], c["pods"], [c["pod"]])
        assert cl.image_locality
        plan = scheduler.plan(cl, [], [("ImageLocalityPriority", 1)])
        cls = int(cl.pods[0]["cls"])
        t = plan.tables
        got = {cl.names[i]: int(plan.na_add[cls][t["na_class"][cls][cl.cols["label_set"][i]]]) + plan.const_score
               for i in range(cl.n_nodes)}
        assert [[h, got[h]] for h, _ in c["expect"]] == c["expect"], c["test"]
        bare = ingest.Cluster.from_objects(c["nodes"], c["pods"], [c["pod"]], image_locality=False)
        with pytest.raises(abi.KsimUnsupported):
            scheduler.plan(bare, [], [("ImageLocalityPriority", 1)])
