"""The C++ Kubernetes-field front end (include/ksim_k8s.h) against the Python host's ingest: the same
Kubernetes-shaped objects flattened into ksim_k8s_* structs (ksim/frontend.py, what a cgo adapter
does) must give the same node table, class tables, pod descriptors, inter-pod affinity tables and
volume tables, array for array — on random workloads exercising every string rule (selectors, node
affinity, tolerations, preferAvoidPods, host ports, scalar resources, affinity terms with
namespaces and topology keys, SelectorSpread listers and zones, every volume kind and the PV / PVC
listers).  CPU only: no device call."""
import ctypes as C

import numpy as np
import pytest

from ksim import abi, frontend, ingest, synth
from ksim.spread import SpreadListers
from workloads import (add_prefer_avoid, rnd_affinity_workload, rnd_mixed_workload, rnd_spread_workload,
                       rnd_volume_workload, rnd_workload)


def _arr(p, n, ctype):
    if n == 0:
        return np.zeros(0)
    return np.ctypeslib.as_array(C.cast(p, C.POINTER(ctype)), shape=(n,)).copy()


def _node_cols(t):
    n, S, P = t.n_nodes, t.n_scalar, t.port_slots
    out = {}
    for name, ct, m in (("alloc_cpu", C.c_int64, 1), ("alloc_mem", C.c_int64, 1), ("alloc_gpu", C.c_int64, 1),
                        ("alloc_eph", C.c_int64, 1), ("allowed_pods", C.c_int32, 1), ("flags", C.c_uint32, 1),
                        ("label_set", C.c_int32, 1), ("taint_set", C.c_int32, 1), ("alloc_scalar", C.c_int64, S),
                        ("req_cpu", C.c_int64, 1), ("req_mem", C.c_int64, 1), ("req_gpu", C.c_int64, 1),
                        ("req_eph", C.c_int64, 1), ("nz_cpu", C.c_int64, 1), ("nz_mem", C.c_int64, 1),
                        ("pod_count", C.c_int32, 1), ("req_scalar", C.c_int64, S), ("ports", C.c_uint64, P),
                        ("port_count", C.c_int32, 1)):
        out[name] = _arr(getattr(t, name), n * m, ct)
    return out


def _compare(cl, fe):
    assert fe.names == cl.names
    nt, ct, at, vt = fe.tables()
    py = cl.node_table()
    assert (nt.n_nodes, nt.n_scalar, nt.port_slots) == (py.n_nodes, py.n_scalar, py.port_slots)
    a, b = _node_cols(nt), _node_cols(py)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    d = cl.tables
    assert (ct.n_classes, ct.n_label_sets, ct.n_taint_sets) == (d["n_classes"], d["n_label_sets"], d["n_taint_sets"])
    assert (ct.val_width or abi.MAX_RCLASS) == d["tt_val"].shape[1] == d["na_val"].shape[1]
    for name, ctype in (("sel_ok", C.c_uint32), ("taint_ok", C.c_uint32), ("noexec_ok", C.c_uint32), ("tt_class", C.c_uint8),
                        ("na_class", C.c_uint8), ("n_tt", C.c_int32), ("n_na", C.c_int32), ("tt_val", C.c_int64),
                        ("na_val", C.c_int64)):
        want = np.ascontiguousarray(d[name]).ravel()
        assert np.array_equal(_arr(getattr(ct, name), want.size, ctype), want), name
    pods, ports, scalars = fe.pods()
    assert len(pods) == len(cl.pods)
    for f in abi.POD_DTYPE.names:
        if f == "reserved":
            continue
        assert np.array_equal(pods[f], cl.pods[f]), f
    assert np.array_equal(ports, cl.pod_ports)
    assert np.array_equal(scalars, cl.pod_scalars)
    if cl.affinity is None:
        assert at.n_nodes == 0
    else:
        A = cl.affinity
        for k in ("n_keys", "n_sel", "n_ident", "n_pair", "n_carry", "n_aclass", "sel_words", "carry_words", "zone_key"):
            assert getattr(at, k) == int(A[k]), k
        assert (at.n_terms, at.n_carries) == (A["n_terms"], A["n_carries"])
        for name, ctype in (("dom", C.c_int32), ("n_dom", C.c_int32), ("ident_sel", C.c_uint64), ("ident_anti", C.c_uint64),
                            ("ident_prio", C.c_uint64), ("pair_sel", C.c_int32), ("pair_key", C.c_int32),
                            ("pair_off", C.c_int64), ("carry_key", C.c_int32), ("carry_kind", C.c_int32),
                            ("carry_off", C.c_int64), ("ac", C.c_int32), ("cnt", C.c_int32), ("carried", C.c_int64),
                            ("spread_pair", C.c_int32)):
            want = np.ascontiguousarray(A[name]).ravel()
            assert np.array_equal(_arr(getattr(at, name), want.size, ctype), want), name
        nt_ = A["n_terms"]
        if nt_:
            got_terms = np.frombuffer((C.c_char * (32 * nt_)).from_address(at.terms), np.dtype(A["terms"].dtype))
            assert np.array_equal(got_terms, A["terms"][:nt_])
        nc = A["n_carries"]
        if nc:
            got_car = np.frombuffer((C.c_char * (16 * nc)).from_address(at.carries), np.dtype(A["carries"].dtype))
            assert np.array_equal(got_car, A["carries"][:nc])
    if cl.volumes is None:
        assert vt.n_nodes == 0
    else:
        V = cl.volumes
        assert (vt.n_keys, vt.n_vclass, vt.n_refs, vt.vol_slots) == (len(V["key_filter"]), len(V["vc"]), len(V["refs"]),
                                                                      V["vol_slots"])
        assert list(vt.max_vols) == list(V["max_vols"])
        assert vt.zone_words == V["zone_words"]
        for name, ctype in (("key_filter", C.c_uint32), ("vc", C.c_int32), ("vc_filter", C.c_uint32),
                            ("slots", C.c_uint64), ("slot_count", C.c_int32)):
            want = np.ascontiguousarray(V[name]).ravel()
            assert np.array_equal(_arr(getattr(vt, name), want.size, ctype), want), name
        want = np.ascontiguousarray(V["zone_ok"]).ravel()
        assert np.array_equal(_arr(vt.zone_ok, want.size, C.c_uint32), want), "zone_ok"
        nr = len(V["refs"])
        got = np.frombuffer((C.c_char * (8 * nr)).from_address(vt.refs), abi.VOL_REF_DTYPE) if nr else np.zeros(0, abi.VOL_REF_DTYPE)
        assert np.array_equal(got, V["refs"])


@pytest.mark.parametrize("seed", range(6))
def test_general_workloads(seed):
    nodes, running, pods = rnd_workload(seed, n_nodes=30, n_pods=90)
    _compare(ingest.Cluster.from_objects(nodes, running, pods), frontend.K8sCluster(nodes, running, pods))


@pytest.mark.parametrize("seed", range(3))
def test_very_wide_reduce_dimension_workloads(seed):
    """More than 16 values in one reduce dimension: value rows wider than 16 (ABI 7) alike."""
    from test_oracle_c_features import very_wide_workload
    nodes, running, pods = very_wide_workload(seed, n_nodes=40, n_pods=80)
    _compare(ingest.Cluster.from_objects(nodes, running, pods), frontend.K8sCluster(nodes, running, pods))


@pytest.mark.parametrize("seed", range(4))
def test_prefer_avoid_workloads(seed):
    nodes, running, pods = rnd_workload(50 + seed, n_nodes=20, n_pods=60)
    add_prefer_avoid(seed, nodes, pods)
    _compare(ingest.Cluster.from_objects(nodes, running, pods), frontend.K8sCluster(nodes, running, pods))


@pytest.mark.parametrize("seed", range(6))
def test_affinity_workloads(seed):
    nodes, running, pods = rnd_affinity_workload(seed, n_nodes=22, n_pods=90)
    for hw in (10, 0, 3):
        _compare(ingest.Cluster.from_objects(nodes, running, pods, hard_weight=hw),
                 frontend.K8sCluster(nodes, running, pods, hard_weight=hw))


@pytest.mark.parametrize("seed,zones,resolvable", [(s, z, r) for s in range(4) for z in (False, True) for r in (False, True)])
def test_volume_workloads(seed, zones, resolvable):
    nodes, running, pods, pvs, pvcs = rnd_volume_workload(seed, zones=zones, resolvable_only=resolvable)
    _compare(ingest.Cluster.from_objects(nodes, running, pods, pvs=pvs, pvcs=pvcs),
             frontend.K8sCluster(nodes, running, pods, pvs=pvs, pvcs=pvcs))


@pytest.mark.parametrize("seed", range(5))
def test_spread_workloads(seed):
    nodes, running, pods, objs = rnd_spread_workload(seed)
    for only in (False, True):
        sp = SpreadListers(**objs)
        _compare(ingest.Cluster.from_objects(nodes, running, pods, spread=sp, spread_services_only=only),
                 frontend.K8sCluster(nodes, running, pods, spread=sp, spread_services_only=only))


@pytest.mark.parametrize("seed", range(2))
def test_mixed_workloads(seed):
    nodes, running, pods, pvs, pvcs, objs = rnd_mixed_workload(seed, n_nodes=60, n_pods=300)
    sp = SpreadListers(**objs)
    _compare(ingest.Cluster.from_objects(nodes, running, pods, pvs=pvs, pvcs=pvcs, spread=sp),
             frontend.K8sCluster(nodes, running, pods, pvs=pvs, pvcs=pvcs, spread=sp))


def test_c2x_objects():
    nodes, pods, pvs, pvcs, services = synth.c2x_objects(400, 1500)
    sp = SpreadListers(services=services)
    _compare(ingest.Cluster.from_objects(nodes, (), pods, pvs=pvs, pvcs=pvcs, spread=sp),
             frontend.K8sCluster(nodes, (), pods, pvs=pvs, pvcs=pvcs, spread=sp))


def test_unsupported_inputs_are_refused():
    nodes, running, pods = rnd_affinity_workload(1, n_nodes=6, n_pods=4)
    bad = dict(pods[0])
    bad["spec"] = dict(bad["spec"], affinity={"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"a": "b"}}, "topologyKey": ""}]}})
    with pytest.raises(abi.KsimUnsupported):
        frontend.K8sCluster(nodes, running, [bad])
    with pytest.raises(abi.KsimUnsupported):
        ingest.Cluster.from_objects(nodes, running, [bad])
    node = dict(nodes[0])
    node["status"] = dict(node["status"], conditions=[{"type": "Ready", "status": "False"},
                                                      {"type": "Ready", "status": "Unknown"}])
    with pytest.raises(abi.KsimUnsupported):
        frontend.K8sCluster([node], (), [])


def test_policy_arguments_refused_with_services():
    """CheckServiceAffinity / serviceAntiAffinity through the C++ front end when the adapter's
    ServiceLister selects pods: refused before any device work (the Python host builds those)."""
    from ksim import abi, frontend, scheduler
    from workloads import rnd_workload
    nodes, running, pods = rnd_workload(2, n_nodes=8, n_pods=10)
    fe = frontend.K8sCluster(nodes, running, pods)
    cfg = scheduler.make_config(["GeneralPredicates", "CheckServiceAffinity"], [("LeastRequestedPriority", 1)])
    with pytest.raises(abi.KsimUnsupported):
        fe.open_policy(cfg, service_affinity=["tier"], services_select_pods=True)
    cfg = scheduler.make_config(["GeneralPredicates", "CheckNodeLabelPresence"], [("LeastRequestedPriority", 1)])
    with pytest.raises(abi.KsimUnsupported):
        fe.open(cfg)   # the predicate's arguments only come through ksim_k8s_open_policy


def test_cache_refuses_label_presence_without_argument():
    """CheckNodeLabelPresence without its Policy labelsPresence argument: the reference fails on it
    (predicates/predicates.go NewNodeLabelPredicate needs the labels), so the C++ scheduler cache
    refuses it as plan() does instead of scheduling without the predicate."""
    from ksim import scheduler
    preds = list(scheduler.DEFAULT_PREDICATES) + ["CheckNodeLabelPresence"]
    with pytest.raises(abi.KsimUnsupported, match="labelsPresence"):
        frontend.K8sCache(preds, [("LeastRequestedPriority", 1)])
