"""GPU parity of tree mode (KSIM_MODE_TREE, csrc/ksim_tree.hip):
incremental per-pod-class selection trees instead of the O(N) scan per pod.  Same bar as the
scan kernels: placements, FitError reason histograms, lastNodeIndex and node state identical
to the C oracle (oracle/cpu_ref.c) on the same inputs.  Tree geometries that only larger
tables reach (levels below the LDS in global memory, 1/2/4 leaves per lane) are forced on small
tables through KSIM_TREE_LDS / KSIM_TREE_M."""
import numpy as np
import pytest

from ksim import abi, scheduler, synth

pytestmark = pytest.mark.gpu

PREDS = list(scheduler.DEFAULT_PREDICATES)
LR_BRA = [("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]


def _ref(cl, preds, prios, first=0, count=None):
    import cpu_ref
    return cpu_ref.run(cl, scheduler.make_config(preds, prios), first, count, threads=8)


def _same_state(g, ref_state):
    s = g.node_state()
    for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count"):
        assert np.array_equal(s[k], ref_state[k]), k


# (nodes, KSIM_TREE_LDS bytes, KSIM_TREE_M): default plans, and global levels forced
GEOMETRIES = [(100_000, None, None), (20_000, None, None), (20_000, 4096, "1"), (20_000, 24_000, "2"),
              (20_000, None, "4"), (3_000, 600, "1"), (777, None, "2")]


@pytest.mark.parametrize("n_nodes,lds,m", GEOMETRIES)
def test_tree_c3_shape_matches_c_oracle(n_nodes, lds, m, monkeypatch):
    """C3-shaped cluster and queue (36 pod classes, LeastRequested + BalancedResourceAllocation)
    in uneven chunks (the trees persist across calls): placements, counter and node state."""
    if lds:
        monkeypatch.setenv("KSIM_TREE_LDS", str(lds))
    if m:
        monkeypatch.setenv("KSIM_TREE_M", m)
    P = 6000
    cl, p, q = synth.config_c3(n_nodes, P)
    g = scheduler.GenericScheduler(cl, p, q, mode=abi.MODE_TREE, collect_reasons=False)
    outs, first = [], 0
    for step in (1, 7, 992, 3000, 2000):
        o, _, st = g.schedule(first, step)
        assert st.mode == abi.MODE_TREE and st.blocks == 1
        outs.append(o)
        first += step
    out = np.concatenate(outs)
    ref, _, ref_state, ref_ctr = _ref(cl, p, q, 0, P)
    assert np.array_equal(out, ref)
    assert g.last_node_index == ref_ctr
    _same_state(g, ref_state)


@pytest.mark.parametrize("lds", [None, 2048])
def test_tree_c1_full_with_fit_errors(lds, monkeypatch):
    """Full C1 (1,500 nodes, 48,020 pods, DefaultProvider) until unschedulable: FitError
    histograms (cached per class between commits) and the 1-fit shortcut near saturation."""
    if lds:
        monkeypatch.setenv("KSIM_TREE_LDS", str(lds))
    cl, p, q = synth.config_c1()
    g = scheduler.GenericScheduler(cl, p, q, mode=abi.MODE_TREE)
    out, reasons, st = g.schedule()
    assert st.mode == abi.MODE_TREE
    ref, ref_reasons, ref_state, ref_ctr = _ref(cl, p, q)
    assert np.array_equal(out, ref)
    failed = out < 0
    assert failed.sum() == 20
    assert np.array_equal(reasons[failed], ref_reasons[failed])
    assert g.last_node_index == ref_ctr
    _same_state(g, ref_state)


@pytest.mark.parametrize("n_nodes", [1, 2, 63, 65, 200])
def test_tree_tiny_clusters_until_full(n_nodes):
    """Clusters of 1..200 nodes filled past capacity (single fits, FitErrors) in tree mode."""
    cpu, mem = synth.c3_nodes(n_nodes, 31)
    pcpu, pmem = synth.c3_pods(40 * n_nodes + 20, 31)
    cl = synth.resource_cluster(["t-%03d" % i for i in range(n_nodes)], cpu, mem, np.full(n_nodes, 30, np.int32),
                                pcpu, pmem)
    g = scheduler.GenericScheduler(cl, PREDS, LR_BRA, mode=abi.MODE_TREE)
    out, reasons, st = g.schedule()
    ref, ref_reasons, _, ref_ctr = _ref(cl, PREDS, LR_BRA)
    assert st.mode == abi.MODE_TREE
    assert np.array_equal(out, ref)
    failed = out < 0
    assert failed.sum() > 0 and np.array_equal(reasons[failed], ref_reasons[failed])
    assert g.last_node_index == ref_ctr


@pytest.mark.parametrize("prios", [[("MostRequestedPriority", 3), ("BalancedResourceAllocation", 2)],
                                   [("LeastRequestedPriority", 5)], [], [("EqualPriority", 1)]],
                         ids=["mr-bra", "lr5", "none", "equal"])
def test_tree_policies(prios):
    """Other map-only policies, including an empty prioritizer list (EqualPriority: every fit
    node ties, pure round robin over the fit set)."""
    cl, _, _ = synth.config_c3(5000, 8000, seed=5)
    g = scheduler.GenericScheduler(cl, PREDS, prios, mode=abi.MODE_TREE)
    out, reasons, st = g.schedule()
    ref, ref_reasons, ref_state, ref_ctr = _ref(cl, PREDS, prios)
    assert st.mode == abi.MODE_TREE
    assert np.array_equal(out, ref)
    assert np.array_equal(reasons[out < 0], ref_reasons[out < 0])
    assert g.last_node_index == ref_ctr
    _same_state(g, ref_state)


def test_tree_interleaved_with_scan_modes():
    """Tree calls after scan-kernel calls on the same handle (the trees are rebuilt from the
    node table whenever another path committed): mixed queue of C2 objects (selectors, ports,
    taints — non-resource-only runs take the AUTO path) against the C oracle."""
    from ksim import ingest
    import cpu_ref
    nodes, pods = synth.c2_objects(900, 20_000)
    cl = ingest.Cluster.from_objects(nodes, (), pods)
    p, q = scheduler.provider("DefaultProvider")
    g = scheduler.GenericScheduler(cl, p, q, mode=abi.MODE_TREE)
    out, reasons, _ = g.schedule()
    ref, ref_reasons, ref_state, ref_ctr = cpu_ref.run(cl, scheduler.make_config(p, q), threads=8)
    assert np.array_equal(out, ref)
    assert np.array_equal(reasons[out < 0], ref_reasons[out < 0])
    assert g.last_node_index == ref_ctr
    _same_state(g, ref_state)


def test_tree_hands_over_at_exactness_bound():
    """Commits that take a node's non-zero memory past 2^48 stop the tree kernel after that pod;
    the general kernel finishes the call and later calls."""
    n, m = 300, 3000
    r = synth.splitmix64(91, n + m)
    alloc_mem = np.full(n, 2 ** 48 - 1, np.int64)
    alloc_cpu = synth._pick(r[:n], [4000, 8000, 16000]).astype(np.int64)
    pcpu = synth._pick(r[n:], [100, 250, 500])
    pmem = synth._pick(r[n:] >> np.uint64(7), [2 ** 30, 2 ** 40, 3 * 2 ** 40])
    cl = synth.resource_cluster(["x-%04d" % i for i in range(n)], alloc_cpu, alloc_mem, np.full(n, 60, np.int32),
                                pcpu, pmem)
    cl.cols["nz_mem"][:] = 2 ** 48 - 5 * 2 ** 40
    g = scheduler.GenericScheduler(cl, PREDS, LR_BRA, mode=abi.MODE_TREE)
    out1, rs1, _ = g.schedule(0, 1500)
    out2, rs2, _ = g.schedule(1500, 1500)
    ref, ref_reasons, ref_state, ref_ctr = _ref(cl, PREDS, LR_BRA)
    assert np.array_equal(np.concatenate([out1, out2]), ref)
    assert np.array_equal(np.concatenate([rs1, rs2]), ref_reasons)
    assert g.last_node_index == ref_ctr
    _same_state(g, ref_state)


def test_tree_c4_million_nodes_prefix():
    """1M nodes (one global level below the LDS): the first 2,000 pods against the C oracle."""
    cl, p, q = synth.config_c4(1_000_000, 4000)
    g = scheduler.GenericScheduler(cl, p, q, mode=abi.MODE_TREE, collect_reasons=False)
    out, _, st = g.schedule(0, 2000)
    assert st.mode == abi.MODE_TREE
    ref, _, ref_state, ref_ctr = _ref(cl, p, q, 0, 2000)
    assert np.array_equal(out, ref)
    assert g.last_node_index == ref_ctr
    _same_state(g, ref_state)
