"""GPU parity of pod classes with more than 16 reduce classes (TaintToleration x NodeAffinity /
NodePreferAvoidPods values, formerly refused): the launch form's wide decision — per block and
class the max map score and its count in global memory, the grid's per class in the last block,
NormalizeReduce over the present classes (reduce.go:29-64), the winners' count for selectHost
(generic_scheduler.go:183-198) and the selected block evaluated again to pick the node.  Against
the object oracle (placements, FitError texts, lastNodeIndex), the per-pod call against the batch,
and a 3,000-node run against the C oracle."""
import numpy as np
import pytest

import ksim_ref as R
from ksim import abi, ingest, scheduler
from test_oracle_c_features import very_wide_workload, wide_workload

pytestmark = pytest.mark.gpu


def _wide_pods(cl, g):
    t = g.tables
    k1 = np.asarray(t["n_tt"]) if g.cfg.weights[abi.W_TAINT_TOL] else 1
    k2 = np.asarray(t["n_na"]) if (g.cfg.weights[abi.W_NODE_AFF] or g.na_add is not None) else 1
    return int(((np.asarray(k1) * np.asarray(k2))[np.asarray(cl.pods["cls"])] > 16).sum())


@pytest.mark.parametrize("mode", [abi.MODE_AUTO, abi.MODE_LAUNCH])
@pytest.mark.parametrize("seed", range(4))
def test_wide_reduce_classes_match_oracle(seed, mode):
    nodes, running, pods = wide_workload(seed)
    preds, prios = scheduler.provider("DefaultProvider")
    want, lni = R.simulate(nodes, running, pods, set(preds), list(prios))
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order)
    g = scheduler.GenericScheduler(cl, preds, prios, mode=mode)
    try:
        assert _wide_pods(cl, g) > 0
        out, reasons, st = g.schedule()
        got = [(cl.pod_names[k], cl.names[w] if w >= 0 else None,
                None if w >= 0 else scheduler.fit_error_message(cl.n_nodes, reasons[k], cl.scalar_names.items))
               for k, w in enumerate(out)]
        assert got == want
        assert g.last_node_index == lni
        assert st.mode == abi.MODE_LAUNCH
    finally:
        g.close()


def test_wide_schedule_one_matches_batch():
    import ctypes as C
    nodes, running, pods = wide_workload(1, n_pods=200)
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order)
    preds, prios = scheduler.provider("DefaultProvider")
    batch = scheduler.GenericScheduler(cl, preds, prios, mode=abi.MODE_LAUNCH)
    one = scheduler.GenericScheduler(cl, preds, prios, mode=abi.MODE_LAUNCH)
    try:
        out, _, _ = batch.schedule()
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


def test_wide_at_scale_matches_c_oracle():
    """3,000 nodes (several blocks per pod; the winners spread over blocks) x 1,000 pods."""
    import cpu_ref
    nodes, running, pods = wide_workload(7, n_nodes=3000, n_pods=1000)
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order)
    preds, prios = scheduler.provider("DefaultProvider")
    p = scheduler.plan(cl, preds, prios)
    want, _, _, ctr, _ = cpu_ref.run(cl, None, threads=8, plan=p)
    g = scheduler.GenericScheduler(cl, preds, prios)
    try:
        assert _wide_pods(cl, g) > 20
        out, _, _ = g.schedule()
        assert (out == want).all(), int((out != want).argmax())
        assert g.last_node_index == ctr
    finally:
        g.close()


@pytest.mark.parametrize("mode", [abi.MODE_AUTO, abi.MODE_LAUNCH])
@pytest.mark.parametrize("seed", range(3))
def test_very_wide_reduce_dimension_matches_oracle(seed, mode):
    """More than 16 values in one reduce dimension (up to 64 NodeAffinity weight sums, 25
    TaintToleration counts; formerly refused): the launch form's wide decision over value rows
    wider than 16 (ABI 7), against the object oracle — placements, FitError text, lastNodeIndex."""
    nodes, running, pods = very_wide_workload(seed)
    preds, prios = scheduler.provider("DefaultProvider")
    want, lni = R.simulate(nodes, running, pods, set(preds), list(prios))
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order)
    g = scheduler.GenericScheduler(cl, preds, prios, mode=mode)
    try:
        assert _wide_pods(cl, g) > 0
        out, reasons, st = g.schedule()
        got = [(cl.pod_names[k], cl.names[w] if w >= 0 else None,
                None if w >= 0 else scheduler.fit_error_message(cl.n_nodes, reasons[k], cl.scalar_names.items))
               for k, w in enumerate(out)]
        assert got == want
        assert g.last_node_index == lni
    finally:
        g.close()


def test_very_wide_at_scale_matches_c_oracle():
    """2,000 nodes x 600 pods with > 16 values in one reduce dimension, against the C oracle."""
    import cpu_ref
    nodes, running, pods = very_wide_workload(5, n_nodes=2000, n_pods=600)
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order)
    preds, prios = scheduler.provider("DefaultProvider")
    p = scheduler.plan(cl, preds, prios)
    assert p.tables["tt_val"].shape[1] > 16
    want, _, _, ctr, _ = cpu_ref.run(cl, None, threads=8, plan=p)
    g = scheduler.GenericScheduler(cl, preds, prios)
    try:
        out, _, _ = g.schedule()
        assert (out == want).all(), int((out != want).argmax())
        assert g.last_node_index == ctr
    finally:
        g.close()
