"""Parity at BASELINE.json's full sizes, where the cluster is no longer empty: the GPU drives the
C3 cluster past saturation (cpu runs out at ~2.85M of the C3 pod distribution), the C4 cluster
through 3,000 pods, and C5's scenarios through their full 5,000 pods — and the C oracle
(oracle/cpu_ref.c, pinned to the object oracle by tests/test_oracle_c.py and
tests/test_oracle_scale.py) continues from the GPU's read-back node state and lastNodeIndex over
the next window.  High-occupancy tails are where fit counts collapse, ties multiply, the 1-fit
shortcut is taken and FitErrors dominate."""
import numpy as np
import pytest

import cpu_ref
from ksim import abi, scheduler, synth

pytestmark = pytest.mark.gpu


def _invariants(cl, out, s):
    """Size-independent checks over a whole run: per-node sums conserved, nothing overcommitted."""
    bound = out >= 0
    assert s["pod_count"].sum() == bound.sum()
    assert s["req_cpu"].sum() == cl.pods["add_cpu"][:len(out)][bound].sum()
    assert s["req_mem"].sum() == cl.pods["add_mem"][:len(out)][bound].sum()
    assert np.array_equal(np.bincount(out[bound], minlength=cl.n_nodes), s["pod_count"])
    assert (s["req_cpu"] <= cl.cols["alloc_cpu"]).all() and (s["req_mem"] <= cl.cols["alloc_mem"]).all()


@pytest.mark.timeout(900)
def test_c3_full_queue_matches_c_oracle():
    """BASELINE configs[2] exactly as bench.py times it: 100,000 nodes, the whole 1,000,000-pod
    queue from the empty cluster in ONE ksim_schedule call (the persistent fast kernel), against the
    C oracle over the same queue on 16 host threads (~100 s): every placement, the counter and the
    final node state."""
    cl, p, q = synth.config_c3(100_000, 1_000_000)
    g = scheduler.GenericScheduler(cl, p, q, collect_reasons=True)
    try:
        out, reasons, st = g.schedule()
        assert st.mode == abi.MODE_PERSISTENT and st.blocks > 1
        s = g.node_state()
        ctr = g.last_node_index
    finally:
        g.close()
    ref, ref_reasons, ref_state, ref_ctr = cpu_ref.run(cl, scheduler.make_config(p, q), 0, 1_000_000, threads=16)
    mism = np.flatnonzero(out != ref)
    assert mism.size == 0, ("first mismatch at pod", int(mism[0]), int(out[mism[0]]), int(ref[mism[0]]), mism.size)
    failed = out < 0
    assert np.array_equal(reasons[failed], ref_reasons[failed])
    assert ctr == ref_ctr
    for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count"):
        assert np.array_equal(s[k], ref_state[k]), k
    _invariants(cl, out, s)


@pytest.mark.timeout(600)  # the tree form's 2.95M-pod head takes ~140 s
@pytest.mark.parametrize("mode", [abi.MODE_AUTO, abi.MODE_TREE], ids=["scan", "tree"])
def test_c3_saturated_tail_matches_c_oracle(mode):
    """C3 (100k nodes): 2,950,000 pods on the GPU (past cpu saturation), then the next 3,000 on
    the GPU and on the C oracle from the GPU's state: placements, FitError histograms, counter,
    final node state."""
    head, tail = 2_950_000, 3000
    cl, p, q = synth.config_c3(100_000, head + tail)
    g = scheduler.GenericScheduler(cl, p, q, mode=mode, collect_reasons=True)
    out_head, _, _ = g.schedule(0, head)
    state, ctr = g.node_state(), g.last_node_index
    _invariants(cl, out_head, state)
    assert (out_head < 0).sum() > 10_000  # saturated: many FitErrors already
    out, reasons, _ = g.schedule(head, tail)
    ref, ref_reasons, ref_state, ref_ctr = cpu_ref.run(cl, scheduler.make_config(p, q), head, tail, threads=16,
                                                       state=state, counter=ctr)
    assert np.array_equal(out, ref)
    failed = out < 0
    assert failed.sum() > tail // 10
    assert np.array_equal(reasons[failed], ref_reasons[failed])
    assert g.last_node_index == ref_ctr
    s = g.node_state()
    for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count"):
        assert np.array_equal(s[k], ref_state[k]), k
    g.close()


@pytest.mark.parametrize("mode", [abi.MODE_AUTO, abi.MODE_TREE], ids=["scan", "tree"])
def test_c4_3000_pods_match_c_oracle(mode):
    """C4 (1M nodes on one device: the streaming form of the fast kernel, or tree mode): 3,000
    pods against the C oracle, node state included."""
    cl, p, q = synth.config_c4(1_000_000, 3000)
    g = scheduler.GenericScheduler(cl, p, q, mode=mode, collect_reasons=False)
    out1, _, _ = g.schedule(0, 1000)
    out2, _, _ = g.schedule(1000, 2000)
    ref, _, ref_state, ref_ctr = cpu_ref.run(cl, scheduler.make_config(p, q), 0, 3000, threads=16)
    assert np.array_equal(np.concatenate([out1, out2]), ref)
    assert g.last_node_index == ref_ctr
    s = g.node_state()
    for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count"):
        assert np.array_equal(s[k], ref_state[k]), k
    g.close()


C5_EXTREMES = [(1, 1, 0), (16, 16, 15), (1, 16, 0), (16, 1, 0), (1, 1, 15), (16, 16, 0), (1, 16, 15), (16, 1, 15),
               (8, 3, 7)]


@pytest.mark.parametrize("form", ["tree", "scan"])
def test_c5_full_pods_weight_extremes(form, monkeypatch):
    """C5 (20k nodes): nine scenarios at the corners of the (wLR, wBRA, wMR) grid, each through
    all 5,000 pods of the sweep, against the C oracle run under that scenario's weights."""
    if form == "scan":
        monkeypatch.setenv("KSIM_SWEEP_SCAN", "1")
    cl, preds, _ = synth.config_c5(20_000, 5000)
    pick = []
    for a, b, m in C5_EXTREMES:
        pri = [("LeastRequestedPriority", a), ("BalancedResourceAllocation", b)]
        if m:
            pri.append(("MostRequestedPriority", m))
        pick.append(pri)
    g = scheduler.GenericScheduler(cl, preds, pick[0], collect_reasons=False)
    out, ctr, st = g.sweep(pick, 0, 5000)
    assert st.mode == (abi.MODE_TREE if form == "tree" else abi.MODE_PERSISTENT)
    for k, pri in enumerate(pick):
        ref, _, _, ref_ctr = cpu_ref.run(cl, scheduler.make_config(preds, pri), 0, 5000, threads=16)
        assert np.array_equal(out[k], ref), pri
        assert int(ctr[k]) == ref_ctr, pri
    g.close()


def _slot_sets(slots, cnt):
    """Per node, the mounted (key, counts) words as a set (slot order is not part of the state)."""
    return [frozenset(int(slots[s, i]) for s in range(int(cnt[i]))) for i in range(len(cnt))]


@pytest.mark.parametrize("n_nodes,n_pods,mode", [(5000, 20_000, abi.MODE_AUTO), (150, 20_000, abi.MODE_AUTO),
                                                  (5000, 20_000, abi.MODE_PERSISTENT)],
                         ids=["c2x_full", "c2x_saturated", "c2x_persistent"])
def test_c2x_matches_c_oracle(n_nodes, n_pods, mode):
    """C2x (BASELINE configs[1]'s cluster plus zones, volumes, services → SelectorSpread and hostname
    anti-affinity): the whole queue on the GPU against the table-level C oracle (pinned to the object
    oracle from the same objects, tests/test_oracle_c_features.py): placements, FitError histograms,
    lastNodeIndex, node state and every node's volume mounts; and a saturated 150-node variant whose
    tail is FitErrors."""
    cl, preds, prios, _ = synth.config_c2x(n_nodes, n_pods)
    g = scheduler.GenericScheduler(cl, preds, prios, mode=mode, collect_reasons=True)
    try:
        out, reasons, _ = g.schedule()
        ref, ref_reasons, ref_state, ref_ctr, extra = cpu_ref.run(cl, None, threads=16, plan=g.plan)
        assert np.array_equal(out, ref)
        failed = out < 0
        if n_nodes == 150:
            assert failed.sum() > n_pods // 10
        assert np.array_equal(reasons[failed], ref_reasons[failed])
        assert g.last_node_index == ref_ctr
        s = g.node_state()
        for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count", "port_count"):
            assert np.array_equal(s[k], ref_state[k]), k
        slots, cnt = g.volume_state()
        assert np.array_equal(cnt, extra["vcount"])
        assert _slot_sets(slots, cnt) == _slot_sets(extra["vslots"], extra["vcount"])
    finally:
        g.close()


def test_pgen_spin_abort_recovers(monkeypatch):
    """The general persistent kernel's spin bounds running out (its grid not co-resident after all):
    KSIM_PGEN_TEST_STALL makes the last workgroup exit at once, as one that never became resident,
    and a 1 ms bound ends the others' first wait.  Every workgroup stops before deciding the pod at
    the cursor; the runtime clears the error and finishes the range with the launch form — the whole
    C2x-shaped queue still equals the C oracle (placements, FitErrors, counter, node state)."""
    monkeypatch.setenv("KSIM_PGEN_TEST_STALL", "1")
    monkeypatch.setenv("KSIM_PGEN_SPIN_TICKS", "100000")
    cl, preds, prios, _ = synth.config_c2x(600, 3000)
    g = scheduler.GenericScheduler(cl, preds, prios, collect_reasons=True)
    try:
        out, reasons, st = g.schedule()
        assert st.mode == abi.MODE_LAUNCH  # finished by the launch form after the abort
        ref, ref_reasons, ref_state, ref_ctr, _ = cpu_ref.run(cl, None, threads=16, plan=g.plan)
        assert np.array_equal(out, ref)
        failed = out < 0
        assert np.array_equal(reasons[failed], ref_reasons[failed])
        assert g.last_node_index == ref_ctr
        s = g.node_state()
        for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count", "port_count"):
            assert np.array_equal(s[k], ref_state[k]), k
    finally:
        g.close()
