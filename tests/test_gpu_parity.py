"""GPU parity: libksim.so (HIP, gfx950) against the CPU oracle and the golden vectors
transcribed from the reference's Go tests.  Bit-exact is the bar for every integer result
(placements, scores, reason histograms, node state, lastNodeIndex)."""
import os

import numpy as np
import pytest

import ksim_ref as R
from golden_util import case_id, load
from ksim import abi, ingest, scheduler
from workloads import add_prefer_avoid, rnd_workload

pytestmark = pytest.mark.gpu

MODES = [abi.MODE_LAUNCH, abi.MODE_AUTO, abi.MODE_TREE]


def _sched(nodes, running, pods, preds, prios, mode=abi.MODE_AUTO, **kw):
    cl = ingest.Cluster.from_objects(nodes, running, pods)
    return cl, scheduler.GenericScheduler(cl, preds, prios, mode=mode, **kw)


@pytest.mark.parametrize("c", load("priorities"), ids=case_id)
def test_golden_priorities_on_gpu(c):
    cl, g = _sched(c["nodes"], c["pods"], [c["pod"]], [], [(c["priority"], 1)])
    idx, total = g.priority_scores(0, over=np.arange(cl.n_nodes))
    got = {cl.names[i]: int(s) for i, s in zip(idx, total)}
    assert [[h, got[h]] for h, _ in c["expect"]] == c["expect"]


REDUCE_PRIORITIES = ("TaintTolerationPriority", "NodeAffinityPriority", "NodePreferAvoidPodsPriority",
                     "ImageLocalityPriority")


@pytest.mark.parametrize("mode", [abi.MODE_LAUNCH, abi.MODE_PERSISTENT])
@pytest.mark.parametrize("c", [c for c in load("priorities") if c["priority"] in REDUCE_PRIORITIES], ids=case_id)
def test_golden_reduce_priorities_select_on_gpu(c, mode):
    """The reference's TaintToleration / NodeAffinity / NodePreferAvoidPods / ImageLocality golden
    vectors through the scheduling kernels' own reduce classes (ImageLocality and NodePreferAvoidPods
    as per-class addends) (per-class maxima, class totals — not the host
    numpy path priority_scores uses): with lastNodeIndex = k, the pod must land on the k-th host
    of the golden maximum in descending bytewise name order (selectHost,
    generic_scheduler.go:183-198), for every k over two periods."""
    expect = dict((h, s) for h, s in c["expect"])
    best = max(expect.values())
    tied = sorted((h for h, s in expect.items() if s == best), key=lambda h: h.encode(), reverse=True)
    for k in range(2 * len(tied)):
        cl, g = _sched(c["nodes"], c["pods"], [c["pod"]], [], [(c["priority"], 1)], mode=mode, last_node_index=k)
        assert cl.n_nodes == len(expect)
        out, _, _ = g.schedule(0, 1)
        assert cl.names[int(out[0])] == tied[k % len(tied)], (k, tied)
        assert g.last_node_index == (k + 1 if len(expect) > 1 else k)
        g.close()


@pytest.mark.parametrize("c", load("predicates"), ids=case_id)
def test_golden_predicates_on_gpu(c):
    cl, g = _sched([c["node"]], c["pods"], [c["pod"]], [c["predicate"]], [("EqualPriority", 1)])
    fit, rs, _, _ = g.evaluate(0)
    assert bool(fit[0]) == c["fits"]
    if not c["fits"] and c["reasons"] is not None:
        got = scheduler.reason_strings(int(rs[0]), cl.scalar_names.items)
        assert sorted(got) == sorted(c["reasons"])


@pytest.mark.parametrize("c", load("prioritize"), ids=case_id)
def test_golden_zero_request_on_gpu(c):
    cl, g = _sched(c["nodes"], c["pods"], [c["pod"]], [], [tuple(x) for x in c["configs"]])
    _, total = g.priority_scores(0, over=np.arange(cl.n_nodes))
    if "expect_all_equal" in c:
        assert all(int(s) == c["expect_all_equal"] for s in total)
    else:
        assert all(int(s) != c["expect_none_equal"] for s in total)


def _oracle_run(nodes, running, pods, preds, prios):
    out, lni = R.simulate(nodes, running, pods, set(preds), list(prios))
    return out, lni


def _gpu_run(nodes, running, pods, preds, prios, mode):
    cc = scheduler.ClusterCapacity(nodes, running, pods, predicates=preds, priorities=prios, mode=mode)
    rep = cc.run()
    got = {}
    for name, host in rep.successful:
        got[name] = (host, None)
    for name, msg in rep.failed:
        got[name] = (None, msg)
    return got, rep


POLICIES = {
    "default": scheduler.provider("DefaultProvider"),
    "talkintdata": scheduler.provider("TalkintDataProvider"),
    "lr_bra": (list(scheduler.DEFAULT_PREDICATES), [("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]),
    "weighted": (["CheckNodeCondition", "PodFitsResources", "PodFitsHostPorts", "MatchNodeSelector", "HostName",
                  "PodToleratesNodeTaints", "CheckNodeMemoryPressure"],
                 [("MostRequestedPriority", 3), ("BalancedResourceAllocation", 2), ("TaintTolerationPriority", 5),
                  ("NodeAffinityPriority", 2)]),
    "equal": (["GeneralPredicates"], []),
}


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("policy", sorted(POLICIES))
@pytest.mark.parametrize("seed", range(4))
def test_simulation_matches_oracle(seed, policy, mode):
    nodes, running, pods = rnd_workload(seed, n_nodes=23 + seed * 17, n_pods=150)
    preds, prios = POLICIES[policy]
    want, want_lni = _oracle_run(nodes, running, pods, preds, prios)
    got, rep = _gpu_run(nodes, running, pods, preds, prios, mode)
    order = [name for name, _, _ in want]
    assert [n for n, _ in rep.successful] == [n for n, h, _ in want if h is not None]  # bind order
    for name, host, msg in want:
        assert got[name] == (host, msg), name
    assert rep.last_node_index == want_lni


PA_POLICIES = {
    "default": scheduler.provider("DefaultProvider"),
    "pa_only": (["GeneralPredicates"], [("NodePreferAvoidPodsPriority", 3)]),
    "pa_affinity": (["GeneralPredicates", "PodToleratesNodeTaints"],
                    [("NodePreferAvoidPodsPriority", 2), ("NodeAffinityPriority", 3), ("TaintTolerationPriority", 1),
                     ("LeastRequestedPriority", 1)]),
}


@pytest.mark.parametrize("mode", [abi.MODE_LAUNCH, abi.MODE_PERSISTENT, abi.MODE_AUTO])
@pytest.mark.parametrize("policy", sorted(PA_POLICIES))
@pytest.mark.parametrize("seed", range(3))
def test_prefer_avoid_matches_oracle(seed, policy, mode):
    """NodePreferAvoidPods with RC / RS-owned pods and preferAvoidPods node annotations (its
    weighted score rides the kernels' NodeAffinity reduce classes, ksim_class_tables.na_add)
    against the object oracle's CalculateNodePreferAvoidPodsPriorityMap."""
    nodes, running, pods = rnd_workload(300 + seed, n_nodes=21 + seed * 11, n_pods=140)
    nodes, pods = add_prefer_avoid(seed, nodes, pods)
    preds, prios = PA_POLICIES[policy]
    want, want_lni = _oracle_run(nodes, running, pods, preds, prios)
    got, rep = _gpu_run(nodes, running, pods, preds, prios, mode)
    assert [n for n, _ in rep.successful] == [n for n, h, _ in want if h is not None]
    for name, host, msg in want:
        assert got[name] == (host, msg), name
    assert rep.last_node_index == want_lni


@pytest.mark.parametrize("mode", MODES)
def test_round_robin_descending_names(mode):
    """Derived pin (no reference test fixes the sequence): identical nodes, identical pods →
    hosts visited in descending bytewise name order with period = number of ties."""
    names = ["n-1", "n-10", "n-2"]
    nodes = [{"metadata": {"name": n}, "status": {"allocatable": {"cpu": "100", "memory": "100Gi", "pods": "100"}}}
             for n in names]
    pods = [{"metadata": {"name": "p%d" % i}, "spec": {"containers": [{}]}} for i in range(6)]
    cc = scheduler.ClusterCapacity(nodes, [], pods, predicates=["GeneralPredicates"], priorities=[("EqualPriority", 1)],
                                   mode=mode)
    rep = cc.run()
    assert [h for _, h in rep.successful] == ["n-2", "n-10", "n-1"] * 2
    assert rep.last_node_index == 6


@pytest.mark.parametrize("mode", MODES)
def test_single_fit_does_not_advance_counter(mode):
    nodes = [{"metadata": {"name": "a"}, "status": {"allocatable": {"cpu": "1", "memory": "1Gi", "pods": "10"}}},
             {"metadata": {"name": "b"}, "status": {"allocatable": {"cpu": "4", "memory": "1Gi", "pods": "10"}}}]
    pods = [{"metadata": {"name": "big"}, "spec": {"containers": [{"resources": {"requests": {"cpu": "2"}}}]}}]
    cc = scheduler.ClusterCapacity(nodes, [], pods, mode=mode)
    rep = cc.run()
    assert rep.successful == [("big", "b")]
    assert rep.last_node_index == 0


@pytest.mark.parametrize("mode", MODES)
def test_readme_shape_small(mode):
    """etc/pod.yaml (A: cpu 1 / mem 1, B: cpu 100 / mem 1000) on test-{i}.test.com nodes,
    default provider, LIFO: the B pods are tried first and fail, then A fills the nodes."""
    n = 60
    nodes = [{"metadata": {"name": "test-%d.test.com" % i},
              "status": {"allocatable": {"cpu": "32", "memory": "128Gi", "pods": "110"},
                         "conditions": [{"type": "Ready", "status": "True"}]}} for i in range(n)]
    spec = [{"name": "A", "num": 32 * n + 5, "pod": {"spec": {"containers": [{"resources": {"requests": {"cpu": 1, "memory": 1}}}]}}},
            {"name": "B", "num": 10, "pod": {"spec": {"containers": [{"resources": {"requests": {"cpu": 100, "memory": 1000}}}]}}}]
    pods = scheduler.expand_simulation_pods(spec)
    preds, prios = scheduler.provider("DefaultProvider")
    want, want_lni = _oracle_run(nodes, [], pods, preds, prios)
    got, rep = _gpu_run(nodes, [], pods, preds, prios, mode)
    assert len(rep.successful) == 32 * n
    for name, host, msg in want:
        assert got[name] == (host, msg), name
    assert rep.last_node_index == want_lni


@pytest.mark.parametrize("mode", MODES)
def test_node_state_after_run(mode):
    nodes, running, pods = rnd_workload(7, n_nodes=40, n_pods=200)
    preds, prios = scheduler.provider("DefaultProvider")
    want, _ = _oracle_run(nodes, running, pods, preds, prios)
    cc = scheduler.ClusterCapacity(nodes, running, pods, predicates=preds, priorities=prios, mode=mode)
    cc.run()
    st = cc.scheduler.node_state()
    infos = {ni.name: ni for ni in [R.NodeInfo(x) for x in nodes]}
    for p in running:
        if p["spec"]["nodeName"] in infos:
            infos[p["spec"]["nodeName"]].add_pod(p)
    byname = {p["metadata"]["name"]: p for p in pods}
    for name, host, _ in want:
        if host:
            infos[host].add_pod(byname[name])
    for i, nm in enumerate(cc.cluster.names):
        ni = infos[nm]
        assert st["req_cpu"][i] == ni.requested.cpu and st["req_mem"][i] == ni.requested.mem
        assert st["nz_cpu"][i] == ni.nonzero_cpu and st["nz_mem"][i] == ni.nonzero_mem
        assert st["pod_count"][i] == len(ni.pods)
        assert st["port_count"][i] == len(ni.used_ports)


@pytest.mark.parametrize("mode", MODES)
def test_c1_full_matches_c_oracle(mode):
    """Full C1 (README shape, 1,500 nodes, 48,020 pods, DefaultProvider) against the C oracle."""
    import cpu_ref
    from ksim import synth
    cl, p, q = synth.config_c1()
    g = scheduler.GenericScheduler(cl, p, q, mode=mode)
    out, reasons, st = g.schedule()
    ref, ref_reasons, ref_state, ref_ctr = cpu_ref.run(cl, scheduler.make_config(p, q), threads=8)
    assert np.array_equal(out, ref)
    assert (out >= 0).sum() == 1500 * 32  # cpu saturates at 32 A pods per node
    failed = out < 0
    assert np.array_equal(reasons[failed], ref_reasons[failed])
    assert g.last_node_index == ref_ctr
    s = g.node_state()
    for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count"):
        assert np.array_equal(s[k], ref_state[k]), k


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("n_nodes", [5000, 900])  # C2 as specified; shrunk so it overflows (FitErrors)
def test_c2_matches_c_oracle(n_nodes, mode):
    """C2 (BASELINE.json configs[1]): heterogeneous nodes, 50,000 pods with nodeSelector, host
    ports, taints / tolerations and BestEffort pods, DefaultProvider, through the object
    ingest path — placements, reason histograms, counter and node state (ports included)
    equal the C oracle's."""
    import cpu_ref
    from ksim import synth
    nodes, pods = synth.c2_objects(n_nodes, 50_000)
    cl = ingest.Cluster.from_objects(nodes, (), pods)
    p, q = scheduler.provider("DefaultProvider")
    g = scheduler.GenericScheduler(cl, p, q, mode=mode)
    out, reasons, _ = g.schedule()
    ref, ref_reasons, ref_state, ref_ctr = cpu_ref.run(cl, scheduler.make_config(p, q), threads=8)
    assert np.array_equal(out, ref)
    failed = out < 0
    assert np.array_equal(reasons[failed], ref_reasons[failed])
    assert g.last_node_index == ref_ctr
    s = g.node_state()
    for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count", "port_count"):
        assert np.array_equal(s[k], ref_state[k]), k
    # port slots hold a set: compare per node as sets
    assert all(set(s["ports"][:, i]) == set(ref_state["ports"][:, i]) for i in range(0, cl.n_nodes, 7))
    assert (failed.sum() > 1000) == (n_nodes < 1000)


@pytest.mark.parametrize("mode", MODES)
def test_c4_million_nodes_prefix_matches_c_oracle(mode):
    """C4 scale on one device (BASELINE.json configs[3]: 1M nodes; the table no longer fits
    on chip, so AUTO takes the HBM-streaming launch mode): the first 400 pods against the C
    oracle."""
    import cpu_ref
    from ksim import synth
    cl, p, q = synth.config_c4(1_000_000, 2000)
    g = scheduler.GenericScheduler(cl, p, q, mode=mode, collect_reasons=False)
    out, _, st = g.schedule(0, 400)
    ref, _, ref_state, ref_ctr = cpu_ref.run(cl, scheduler.make_config(p, q), 0, 400, threads=8)
    assert np.array_equal(out, ref)
    assert g.last_node_index == ref_ctr
    s = g.node_state()
    for k in ("req_cpu", "req_mem", "pod_count"):
        assert np.array_equal(s[k], ref_state[k]), k


@pytest.mark.parametrize("mode", MODES)
def test_c3_prefix_matches_c_oracle(mode):
    """100k-node C3 cluster: the first 3,000 pods against the C oracle, then size-independent
    invariants over 60,000 pods (every pod bound, per-node sums conserved)."""
    import cpu_ref
    from ksim import synth
    cl, p, q = synth.config_c3(100_000, 60_000)
    g = scheduler.GenericScheduler(cl, p, q, mode=mode, collect_reasons=False)
    out1, _, _ = g.schedule(0, 3000)
    ref, _, _, ref_ctr = cpu_ref.run(cl, scheduler.make_config(p, q), 0, 3000, threads=8)
    assert np.array_equal(out1, ref)
    assert g.last_node_index == ref_ctr
    out2, _, _ = g.schedule(3000, 57000)
    out = np.concatenate([out1, out2])
    assert (out >= 0).all()
    s = g.node_state()
    assert s["pod_count"].sum() == 60000
    assert s["req_cpu"].sum() == cl.pods["add_cpu"].sum()
    assert s["req_mem"].sum() == cl.pods["add_mem"].sum()
    assert np.array_equal(np.bincount(out, minlength=cl.n_nodes), s["pod_count"])
    assert (s["req_cpu"] <= cl.cols["alloc_cpu"]).all() and (s["req_mem"] <= cl.cols["alloc_mem"]).all()


def test_wave_dpp_selftest():
    """DPP wave reductions / prefix scan used by the persistent kernel vs plain lane loops."""
    assert abi.lib().ksim_selftest() == 0


BOUNDARY_ALLOC = [0, 1, 3, 7, 10, 999, 1000, 1001, 2 ** 20 + 1, 3 * 2 ** 30, 2 ** 48 - 1, 2 ** 48 + 12345,
                  2 ** 49 - 1, 2 ** 49, 2 ** 50 + 7, 10 ** 15 + 3]
BOUNDARY_REQ = [0, 1, 2, 3, 7, 100, 333, 1000, 2 ** 20, 2 ** 30 + 1, 2 ** 40, 2 ** 47, 2 ** 48 + 1]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("prios", [[("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)],
                                   [("MostRequestedPriority", 2), ("LeastRequestedPriority", 1),
                                    ("BalancedResourceAllocation", 3)]], ids=["lr_bra", "mr_lr_bra"])
def test_score_boundaries_match_c_oracle(prios, mode):
    """Resource-only pods on capacities around the fast path's exactness bounds (2^49, exact
    multiples, request == capacity, zero capacity): every placement, reason histogram and the
    final node state equal the C oracle's."""
    import cpu_ref
    from ksim import synth
    n, m = 700, 2500
    r = synth.splitmix64(77, 2 * n + 2 * m)
    cpu = synth._pick(r[0:n], BOUNDARY_ALLOC)
    mem = synth._pick(r[n:2 * n], BOUNDARY_ALLOC)
    pcpu = synth._pick(r[2 * n:2 * n + m], BOUNDARY_REQ)
    pmem = synth._pick(r[2 * n + m:], BOUNDARY_REQ)
    names = ["b-%05d" % i for i in range(n)]
    cl = synth.resource_cluster(names, cpu, mem, np.full(n, 40, np.int32), pcpu, pmem)
    preds = list(scheduler.DEFAULT_PREDICATES)
    g = scheduler.GenericScheduler(cl, preds, prios, mode=mode)
    out, reasons, _ = g.schedule()
    ref, ref_reasons, ref_state, ref_ctr = cpu_ref.run(cl, scheduler.make_config(preds, prios), threads=8)
    assert np.array_equal(out, ref)
    assert np.array_equal(reasons, ref_reasons)
    assert g.last_node_index == ref_ctr
    s = g.node_state()
    for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count"):
        assert np.array_equal(s[k], ref_state[k]), k
    assert (out >= 0).sum() > m // 4  # the queue is not all FitErrors


def test_fast_kernel_hands_over_at_exactness_bound():
    """Resource-only pods whose commits take nodes' non-zero requested memory past 2^48: the
    specialised float64 kernel (ksim_pfast.hip) stops before the next pod and the general
    kernel finishes the call — placements, histograms, counter and node state equal the C
    oracle's, and a later call (general kernel from the start) still agrees."""
    import cpu_ref
    from ksim import synth
    n, m = 300, 3000
    r = synth.splitmix64(91, n + m)
    alloc_mem = np.full(n, 2 ** 48 - 1, np.int64)
    alloc_cpu = synth._pick(r[:n], [4000, 8000, 16000]).astype(np.int64)
    pcpu = synth._pick(r[n:], [100, 250, 500])
    pmem = synth._pick(r[n:] >> np.uint64(7), [2 ** 30, 2 ** 40, 3 * 2 ** 40])
    names = ["x-%04d" % i for i in range(n)]
    cl = synth.resource_cluster(names, alloc_cpu, alloc_mem, np.full(n, 60, np.int32), pcpu, pmem)
    cl.cols["nz_mem"][:] = 2 ** 48 - 5 * 2 ** 40  # already close to the bound
    preds = list(scheduler.DEFAULT_PREDICATES)
    prios = [("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]
    g = scheduler.GenericScheduler(cl, preds, prios)
    out1, rs1, _ = g.schedule(0, 1500)
    out2, rs2, _ = g.schedule(1500, 1500)
    ref, ref_reasons, ref_state, ref_ctr = cpu_ref.run(cl, scheduler.make_config(preds, prios), threads=8)
    assert np.array_equal(np.concatenate([out1, out2]), ref)
    assert np.array_equal(np.concatenate([rs1, rs2]), ref_reasons)
    assert g.last_node_index == ref_ctr
    s = g.node_state()
    for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count"):
        assert np.array_equal(s[k], ref_state[k]), k
    assert s["nz_mem"].max() >= 2 ** 48  # the bound was actually crossed


@pytest.mark.parametrize("seed", [3, 8])
def test_fast_and_general_kernels_agree(seed, monkeypatch):
    """The same resource-only queue through the specialised kernel and, with KSIM_NO_PFAST, the
    general persistent kernel: identical placements, counter and node state (and both equal
    the C oracle's)."""
    import cpu_ref
    from ksim import synth
    res = []
    for env in (None, "1"):
        if env:
            monkeypatch.setenv("KSIM_NO_PFAST", env)
        cl, p, q = synth.config_c3(30_000, 4000, seed=seed)
        g = scheduler.GenericScheduler(cl, p, q, mode=abi.MODE_PERSISTENT, collect_reasons=False)
        out, _, _ = g.schedule(0, 4000)
        res.append((out, g.last_node_index, g.node_state()))
        monkeypatch.delenv("KSIM_NO_PFAST", raising=False)
    (o1, c1, s1), (o2, c2, s2) = res
    assert np.array_equal(o1, o2) and c1 == c2
    for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count"):
        assert np.array_equal(s1[k], s2[k]), k
    ref, _, _, ref_ctr = cpu_ref.run(cl, scheduler.make_config(p, q), 0, 4000, threads=8)
    assert np.array_equal(o1, ref) and c1 == ref_ctr


SWEEP_FORMS = ["tree", "tree-chunked", "scan"]


def _sweep_form(form, monkeypatch):
    """tree: one tree-mode wave per scenario (ksim_tree.hip); scan: the per-scenario scan kernel
    (ksim_sweep.hip); tree-chunked: scenarios in launches of 5."""
    if form == "scan":
        monkeypatch.setenv("KSIM_SWEEP_SCAN", "1")
    if form == "tree-chunked":
        monkeypatch.setenv("KSIM_SWEEP_CHUNK", "5")
    return abi.MODE_PERSISTENT if form == "scan" else abi.MODE_TREE


@pytest.mark.parametrize("form", SWEEP_FORMS)
@pytest.mark.parametrize("n_nodes,n_pods", [(1500, 1200), (20_000, 300)])
def test_sweep_matches_c_oracle_per_scenario(n_nodes, n_pods, form, monkeypatch):
    """Scenario sweep (C5 shape): every scenario's placements and final lastNodeIndex equal the
    C oracle run under that scenario's weights; the scheduler's own state is untouched."""
    import cpu_ref
    from ksim import synth
    mode = _sweep_form(form, monkeypatch)
    cl, preds, scen = synth.config_c5(n_nodes, n_pods)
    pick = [scen[i] for i in (0, 1, 17, 255, 256, 1000, 2047, 2500, 3071, 4095)]
    pick.append([("MostRequestedPriority", 1)])
    pick.append([("LeastRequestedPriority", 7)])
    g = scheduler.GenericScheduler(cl, preds, scen[0], collect_reasons=False)
    before = g.node_state()
    out, ctr, st = g.sweep(pick, 0, n_pods)
    assert st.node_evals == len(pick) * n_pods * n_nodes
    assert st.mode == mode
    for k, pri in enumerate(pick):
        ref, _, _, ref_ctr = cpu_ref.run(cl, scheduler.make_config(preds, pri), 0, n_pods, threads=8)
        assert np.array_equal(out[k], ref), pri
        assert int(ctr[k]) == ref_ctr, pri
    after = g.node_state()
    for k in before:
        assert np.array_equal(before[k], after[k]), k
    assert g.last_node_index == 0


@pytest.mark.parametrize("form", SWEEP_FORMS)
def test_sweep_until_unschedulable_and_from_mid_queue(form, monkeypatch):
    """A sweep over a queue that overflows a small cluster (FitErrors, single-fit pods) started
    after a regular ksim_schedule prefix: continues from the scheduled state and counter."""
    import cpu_ref
    from ksim import synth
    _sweep_form(form, monkeypatch)
    n = 64
    cpu, mem = synth.c3_nodes(n, 11)
    pcpu, pmem = synth.c3_pods(3000, 11)
    cl = synth.resource_cluster(["s-%03d" % i for i in range(n)], cpu, mem, np.full(n, 30, np.int32), pcpu, pmem)
    preds = list(scheduler.DEFAULT_PREDICATES)
    base = [("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]
    g = scheduler.GenericScheduler(cl, preds, base, collect_reasons=False)
    g.schedule(0, 500)
    pick = [base, [("MostRequestedPriority", 2), ("BalancedResourceAllocation", 1)], [("LeastRequestedPriority", 3)]]
    out, ctr, _ = g.sweep(pick, 500, 2500)
    # reference: the same 500-pod prefix under the base policy, then each scenario's policy
    _, _, state0, ctr0 = cpu_ref.run(cl, scheduler.make_config(preds, base), 0, 500, threads=4)
    for k, pri in enumerate(pick):
        state = {key: v.copy() for key, v in state0.items()}
        ref, _, _, ref_ctr = cpu_ref.run(cl, scheduler.make_config(preds, pri), 500, 2500, threads=4, state=state,
                                         counter=ctr0)
        assert np.array_equal(out[k], ref), pri
        assert int(ctr[k]) == ref_ctr
    assert (out < 0).any()  # the cluster fills up


def _run_sharded_threads(cl, preds, prios, world, ranges, collect_reasons=False, reasons_out=None):
    """world ranks of a node-sharded scheduler on this one device, driven from threads (the
    kernels of all ranks must be co-resident: KSIM_MAX_GRID limits each to 256/world CUs)."""
    import threading
    scheds = [scheduler.ShardedScheduler(cl, preds, prios, r, world, collect_reasons=collect_reasons)
              for r in range(world)]
    scheduler.connect_local_world(scheds)
    outs = [[] for _ in range(world)]
    rs = [[] for _ in range(world)]
    for first, count in ranges:
        errs = []

        def go(r):
            try:
                o, re, _ = scheds[r].schedule(first, count)
                outs[r].append(o)
                rs[r].append(re)
            except Exception as e:  # noqa: BLE001 — surfaced below
                errs.append(e)
        ts = [threading.Thread(target=go, args=(r,)) for r in range(world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errs, errs
    merged = scheduler.merge_sharded([np.concatenate(o) for o in outs])
    if reasons_out is not None:
        reasons_out.append(scheduler.merge_sharded_reasons([np.concatenate(r) for r in rs]))
    return scheds, merged


@pytest.mark.parametrize("world", [2, 3])  # co-resident kernels need a HW queue each (GPU_MAX_HW_QUEUES=4)
def test_node_sharded_in_process_matches_c_oracle(world, monkeypatch):
    """One cluster split into `world` contiguous name-rank shards, one persistent kernel per
    shard exchanging per-pod aggregates through each other's exchange buffers: the merged
    placements, every rank's counter and the per-shard node state equal the C oracle's
    unsharded run (two calls, so the exchange tags run across calls)."""
    import cpu_ref
    from ksim import synth
    monkeypatch.setenv("KSIM_MAX_GRID", str(256 // world // 2))
    cl, p, q = synth.config_c3(40_000, 3000, seed=5)
    scheds, merged = _run_sharded_threads(cl, p, q, world, [(0, 1700), (1700, 1300)])
    ref, _, ref_state, ref_ctr = cpu_ref.run(cl, scheduler.make_config(p, q), 0, 3000, threads=8)
    assert np.array_equal(merged, ref)
    for s in scheds:
        assert s.last_node_index == ref_ctr
        st = s.node_state()
        for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count"):
            assert np.array_equal(st[k], ref_state[k][s.lo:s.hi]), k


def test_node_sharded_fills_cluster_with_fit_errors(monkeypatch):
    """Sharded run over a queue that overflows the cluster: single-fit pods (no counter
    increment), FitErrors on every rank, uneven shard sizes."""
    import cpu_ref
    from ksim import synth
    monkeypatch.setenv("KSIM_MAX_GRID", "40")
    n = 301
    cpu, mem = synth.c3_nodes(n, 13)
    pcpu, pmem = synth.c3_pods(9000, 13)
    cl = synth.resource_cluster(["f-%04d" % i for i in range(n)], cpu, mem, np.full(n, 12, np.int32), pcpu, pmem)
    preds = list(scheduler.DEFAULT_PREDICATES)
    prios = [("LeastRequestedPriority", 2), ("BalancedResourceAllocation", 1)]
    scheds, merged = _run_sharded_threads(cl, preds, prios, 3, [(0, 9000)])
    ref, _, _, ref_ctr = cpu_ref.run(cl, scheduler.make_config(preds, prios), 0, 9000, threads=8)
    assert np.array_equal(merged, ref)
    assert (ref < 0).sum() > 1000
    assert all(s.last_node_index == ref_ctr for s in scheds)


@pytest.mark.parametrize("prios", [[("LeastRequestedPriority", 2), ("BalancedResourceAllocation", 1)],
                                   [("LeastRequestedPriority", 1), ("NodeAffinityPriority", 1), ("TaintTolerationPriority", 1)]],
                         ids=["fast", "reduce"])
def test_node_sharded_fit_errors_match_c_oracle(prios, monkeypatch):
    """FitError when node-sharded: every rank collects the reason histogram of its own shard for
    the pods no node of the world fits, and their sum is the FitError histogram over all nodes
    (generic_scheduler.go:51-90, 289-378) — placements, merged histograms and the FitError text
    ("0/N nodes are available: ...") equal the C oracle's unsharded run, through the fast kernel
    and the launch form's exchange (reduce priorities)."""
    import cpu_ref
    from ksim import synth
    monkeypatch.setenv("KSIM_MAX_GRID", "40")
    n = 301
    cpu, mem = synth.c3_nodes(n, 17)
    pcpu, pmem = synth.c3_pods(6000, 17)
    cl = synth.resource_cluster(["s-%04d" % i for i in range(n)], cpu, mem, np.full(n, 12, np.int32), pcpu, pmem)
    preds = list(scheduler.DEFAULT_PREDICATES)
    got = []
    scheds, merged = _run_sharded_threads(cl, preds, prios, 3, [(0, 3500), (3500, 2500)], collect_reasons=True,
                                          reasons_out=got)
    ref, ref_reasons, _, ref_ctr = cpu_ref.run(cl, scheduler.make_config(preds, prios), threads=8)
    assert np.array_equal(merged, ref)
    assert (ref < 0).sum() > 500
    fail = ref < 0
    assert np.array_equal(got[0][fail], ref_reasons[fail])
    for k in np.nonzero(fail)[0][:50]:
        assert scheduler.fit_error_message(n, got[0][k]) == scheduler.fit_error_message(n, ref_reasons[k])
    assert all(s.last_node_index == ref_ctr for s in scheds)


def _sharded_processes(tmp_path, world, skew, n_nodes, n_pods, split, env_extra=None, wait=150, workload="c3"):
    """`world` shard_worker.py processes over a gloo group; returns their .npz results."""
    import socket
    import subprocess
    import sys
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ)
    env.update(env_extra or {})
    worker = os.path.join(os.path.dirname(__file__), "shard_worker.py")
    procs = [subprocess.Popen([sys.executable, worker, str(r), str(world), str(port), str(tmp_path / ("r%d.npz" % r)),
                               str(skew), str(n_nodes), str(n_pods), str(split), workload], env=env)
             for r in range(world)]
    try:
        rcs = [pr.wait(timeout=wait) for pr in procs]
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
    assert rcs == [0] * world
    return [np.load(tmp_path / ("r%d.npz" % r)) for r in range(world)]


def _check_sharded(res, n_nodes, n_pods, threads=8, workload="c3"):
    import cpu_ref
    from ksim import synth
    if workload == "c3":
        cl, p, q = synth.config_c3(n_nodes, n_pods, seed=9)
        ref, _, ref_state, ref_ctr = cpu_ref.run(cl, scheduler.make_config(p, q), 0, n_pods, threads=threads)
    else:
        cl, p, q = synth.config_c2(n_nodes, n_pods, seed=9) if workload == "c2" else \
            synth.config_c2x(n_nodes, n_pods, seed=9)[:3]
        ref, _, ref_state, ref_ctr, _ = cpu_ref.run(cl, None, threads=threads, plan=scheduler.plan(cl, p, q))
    assert np.array_equal(scheduler.merge_sharded([r["out"] for r in res]), ref)
    assert sum(int(r["hi"]) - int(r["lo"]) for r in res) == n_nodes
    for r in res:
        assert int(r["ctr"]) == ref_ctr
        lo, hi = int(r["lo"]), int(r["hi"])
        for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count"):
            assert np.array_equal(r[k], ref_state[k][lo:hi]), k


@pytest.mark.parametrize("world,skew", [(2, 0.0), (2, 3.5), (4, 0.0), (8, 0.0)])
def test_node_sharded_multi_process(tmp_path, world, skew):
    """`world` ranks in as many processes (the one-process-per-device layout: rank r on device
    r % device_count — all on device 0 of a one-GPU box, each process with its own hardware
    queues), exchange buffers shared through hipIpcGetMemHandle / hipIpcOpenMemHandle over a gloo
    group: merged placements, counters and node state equal the C oracle's.  world = 8 is
    KSIM_MAX_RANKS: every exchange slot and the decision's rank walk at full width.  skew: the
    last rank starts its first call 3.5 s late — beyond the 2 s per-pod spin bound — which the
    first pod's start handshake must absorb."""
    import torch
    env = {}
    if torch.cuda.device_count() < world:  # ranks share a device: their persistent grids must co-reside
        env["KSIM_MAX_GRID"] = str(256 // world // 2)
    res = _sharded_processes(tmp_path, world, skew, 40_000, 2500, 1200, env)
    _check_sharded(res, 40_000, 2500)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_node_sharded_c2_multi_process(tmp_path, world):
    """Node-sharded scheduling of C2-shaped pods (node selectors, required node affinity, taints,
    TaintToleration / NodeAffinity reduce classes) — SURVEY.md §8e Phase A in the launch form:
    each rank's last block exchanges its fit count and per-class (max, count) with every rank, all
    decide on the world's NormalizeReduce maxima and selectHost index, and the rank holding the
    node commits it.  `world` processes on this box's devices; placements, counters and every
    shard's node state equal the C oracle's unsharded run (two calls: tags run across calls)."""
    res = _sharded_processes(tmp_path, world, 0.0, 6000, 800, 300, workload="c2")
    _check_sharded(res, 6000, 800, workload="c2")


@pytest.mark.parametrize("world", [2, 4])
def test_node_sharded_c2x_multi_process(tmp_path, world):
    """Node-sharded C2x (zones, volumes, SelectorSpread over services, required anti-affinity on
    kubernetes.io/hostname): every counted pair and carried term is node-like, so each rank keeps
    the global count arrays over its own nodes' domains and commits on its own rank only; pass A's
    InterPodAffinity min / max, SelectorSpread max / haveZones and zone sums are exchanged across
    the ranks before the scores.  Placements, counters and node state equal the C oracle's."""
    res = _sharded_processes(tmp_path, world, 0.0, 4000, 600, 250, workload="c2x")
    _check_sharded(res, 4000, 600, workload="c2x")


def test_node_sharded_refuses_shared_domains():
    """Terms over topology domains several nodes share (a zone-keyed preferred term) are refused."""
    from workloads import rnd_affinity_workload
    nodes, running, pods = rnd_affinity_workload(1, n_nodes=20, n_pods=40)
    cl = ingest.Cluster.from_objects(nodes, running, pods)
    with pytest.raises(abi.KsimUnsupported):
        cl.shard(0, 10)


def test_node_sharded_c2_in_process_matches_c_oracle():
    """Two ranks of the C2 shape driven from threads of one process (one stream each)."""
    import cpu_ref
    from ksim import synth
    cl, p, q = synth.config_c2(3000, 400, seed=11)
    scheds, merged = _run_sharded_threads(cl, p, q, 2, [(0, 150), (150, 250)])
    ref, _, ref_state, ref_ctr, _ = cpu_ref.run(cl, None, threads=8, plan=scheduler.plan(cl, p, q))
    assert np.array_equal(merged, ref)
    for s in scheds:
        assert s.last_node_index == ref_ctr
        st = s.node_state()
        for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count"):
            assert np.array_equal(st[k], ref_state[k][s.lo:s.hi]), k


@pytest.mark.timeout(600)
def test_node_sharded_c4_shape_world8(tmp_path):
    """C4's real shard shape (BASELINE configs[3]: 1,000,000 nodes over 8 ranks = 125,000 name-rank
    rows per shard), 3,000 pods in two calls, 8 processes.  On a one-GPU box all ranks share device
    0: each rank's grid is capped at 32 workgroups (8 x 32 = every CU, one 512-thread workgroup per
    CU), so every shard takes the streaming form at 3,907 rows per workgroup; on an 8-GPU node each
    rank owns a device.  Placements, counters and every shard's node state equal the C oracle's."""
    import torch
    env = {"KSIM_SHARD_START_S": "60"}
    if torch.cuda.device_count() < 8:
        env["KSIM_MAX_GRID"] = "32"
    res = _sharded_processes(tmp_path, 8, 0.0, 1_000_000, 3000, 1700, env, wait=300)
    _check_sharded(res, 1_000_000, 3000, threads=16)


@pytest.mark.parametrize("max_grid", [0, 128, 64, 28])  # rows per row thread: 1, 2, 4, 9
def test_stream_form_matches_c_oracle(max_grid, monkeypatch):
    """The streaming form of the fast kernel (rows read from the HBM float64 image every pod,
    only the evaluations in LDS — the form for tables beyond the LDS budget, forced here at
    100k nodes with every row-per-thread instantiation): two calls of a C3 prefix equal the C
    oracle, node state included."""
    import cpu_ref
    from ksim import synth
    monkeypatch.setenv("KSIM_FORCE_STREAM", "1")
    if max_grid:
        monkeypatch.setenv("KSIM_MAX_GRID", str(max_grid))
    cl, p, q = synth.config_c3(100_000, 5000, seed=8)
    g = scheduler.GenericScheduler(cl, p, q, collect_reasons=False)
    out1, _, st = g.schedule(0, 2200)
    assert st.mode == abi.MODE_PERSISTENT
    out2, _, _ = g.schedule(2200, 2800)
    ref, _, ref_state, ref_ctr = cpu_ref.run(cl, scheduler.make_config(p, q), 0, 5000, threads=8)
    assert np.array_equal(np.concatenate([out1, out2]), ref)
    assert g.last_node_index == ref_ctr
    s = g.node_state()
    for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count"):
        assert np.array_equal(s[k], ref_state[k]), k


def test_stream_form_fills_cluster_with_fit_errors(monkeypatch):
    """Streaming form over a queue that overflows the cluster: FitError reason histograms,
    single-fit pods (no counter increment), pressure / NotReady nodes."""
    import cpu_ref
    from ksim import synth
    monkeypatch.setenv("KSIM_FORCE_STREAM", "1")
    n = 997
    cpu, mem = synth.c3_nodes(n, 21)
    pcpu, pmem = synth.c3_pods(30_000, 21)
    pcpu[::11] = 0  # some BestEffort-shaped pods (no requests)
    pmem[::11] = 0
    cl = synth.resource_cluster(["s-%05d" % i for i in range(n)], cpu, mem, np.full(n, 25, np.int32), pcpu, pmem)
    cl.pods["flags"][::11] |= abi.POD_BEST_EFFORT
    cl.pods["nz_cpu"][::11] = 100           # non-zero defaults (priorities/util/non_zero.go:31-33)
    cl.pods["nz_mem"][::11] = 200 * 1024 * 1024
    cl.cols["flags"][::37] |= abi.N_MEM_PRESSURE
    cl.cols["flags"][5::101] |= abi.N_NOT_READY
    preds, prios = scheduler.provider("DefaultProvider")
    g = scheduler.GenericScheduler(cl, preds, prios)
    out, reasons, _ = g.schedule()
    ref, ref_reasons, _, ref_ctr = cpu_ref.run(cl, scheduler.make_config(preds, prios), threads=8)
    assert np.array_equal(out, ref)
    failed = out < 0
    assert failed.sum() > 1000
    assert np.array_equal(reasons[failed], ref_reasons[failed])
    assert g.last_node_index == ref_ctr


@pytest.mark.parametrize("world", [2, 3])
def test_node_sharded_stream_form_matches_c_oracle(world, monkeypatch):
    """Node-sharded run whose shards use the streaming form (the 2- and 4-GPU layout of C4)."""
    import cpu_ref
    from ksim import synth
    monkeypatch.setenv("KSIM_FORCE_STREAM", "1")
    monkeypatch.setenv("KSIM_MAX_GRID", str(256 // world // 2))
    cl, p, q = synth.config_c3(60_000, 3000, seed=15)
    scheds, merged = _run_sharded_threads(cl, p, q, world, [(0, 1000), (1000, 2000)])
    ref, _, ref_state, ref_ctr = cpu_ref.run(cl, scheduler.make_config(p, q), 0, 3000, threads=8)
    assert np.array_equal(merged, ref)
    for s in scheds:
        assert s.last_node_index == ref_ctr
        st = s.node_state()
        for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count"):
            assert np.array_equal(st[k], ref_state[k][s.lo:s.hi]), k


# ----------------------------------------------------------------------------- edge cases
def test_no_nodes_is_err_no_nodes_available():
    """genericScheduler.Schedule with an empty node list returns ErrNoNodesAvailable
    (core/generic_scheduler.go:63-64,125): the empty table loads, scheduling on it returns
    KSIM_E_NO_NODES with that text; the simulator's Update records every pod as failed with it
    (simulator.go:163-185) and the last failure writes the capital-F stop reason."""
    pods = [{"metadata": {"name": "p%d" % i}, "spec": {"containers": [{}]}} for i in range(2)]
    cc = scheduler.ClusterCapacity([], [], pods)
    with pytest.raises(abi.NoNodesAvailable) as ei:
        cc.scheduler.schedule()
    assert "no nodes available to schedule pods" in str(ei.value)
    rep = cc.run()
    assert rep.successful == [] and [m for _, m in rep.failed] == ["no nodes available to schedule pods"] * 2
    assert rep.stop_reason == "Fail to get next pod: No pods left\n"
    assert [p["reason"] for p in rep.review["review"]["failed"]["status"]["pods"]] == ["Unschedulable"] * 2


@pytest.mark.parametrize("mode", MODES)
def test_empty_queue_and_empty_ranges(mode):
    """No simulation pods: an empty report and an untouched counter; zero-length and
    out-of-range schedule calls."""
    nodes = [{"metadata": {"name": "n-%d" % i}, "status": {"allocatable": {"cpu": "4", "memory": "8Gi", "pods": "10"}}}
             for i in range(5)]
    rep = scheduler.ClusterCapacity(nodes, [], [], mode=mode).run()
    assert rep.successful == [] and rep.failed == [] and rep.last_node_index == 0
    pods = [{"metadata": {"name": "p%d" % i}, "spec": {"containers": [{}]}} for i in range(3)]
    cc = scheduler.ClusterCapacity(nodes, [], pods, mode=mode)
    out, _, st = cc.scheduler.schedule(1, 0)
    assert len(out) == 0 and st.pods == 0
    with pytest.raises(abi.KsimError):
        cc.scheduler.schedule(2, 5)
    assert cc.scheduler.last_node_index == 0


@pytest.mark.parametrize("n_nodes", [1, 2, 63, 65])
@pytest.mark.parametrize("force_stream", [False, True])
def test_tiny_clusters_fast_kernel(n_nodes, force_stream, monkeypatch):
    """Clusters smaller than one workgroup's rows (a single workgroup, partial waves) in both
    forms of the fast kernel, filled past capacity, against the C oracle."""
    import cpu_ref
    from ksim import synth
    if force_stream:
        monkeypatch.setenv("KSIM_FORCE_STREAM", "1")
    cpu, mem = synth.c3_nodes(n_nodes, 31)
    pcpu, pmem = synth.c3_pods(40 * n_nodes + 20, 31)
    cl = synth.resource_cluster(["t-%03d" % i for i in range(n_nodes)], cpu, mem, np.full(n_nodes, 30, np.int32),
                                pcpu, pmem)
    preds = list(scheduler.DEFAULT_PREDICATES)
    prios = [("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]
    g = scheduler.GenericScheduler(cl, preds, prios)
    out, reasons, st = g.schedule()
    ref, ref_reasons, _, ref_ctr = cpu_ref.run(cl, scheduler.make_config(preds, prios), threads=2)
    assert st.mode == abi.MODE_PERSISTENT
    assert np.array_equal(out, ref)
    failed = out < 0
    assert failed.sum() > 0 and np.array_equal(reasons[failed], ref_reasons[failed])
    assert g.last_node_index == ref_ctr


def test_single_node_fit_error_message():
    """One node, a pod that does not fit: the FitError text (core/generic_scheduler.go:72-90)."""
    nodes = [{"metadata": {"name": "only"}, "status": {"allocatable": {"cpu": "1", "memory": "1Gi", "pods": "5"}}}]
    pods = [{"metadata": {"name": "big"}, "spec": {"containers": [{"resources": {"requests": {"cpu": "2", "memory": "2Gi"}}}]}}]
    rep = scheduler.ClusterCapacity(nodes, [], pods).run()
    assert rep.failed == [("big", "0/1 nodes are available: 1 Insufficient cpu, 1 Insufficient memory.")]


@pytest.mark.parametrize("seed", range(3))
def test_mixed_features_at_scale(seed, monkeypatch):
    """Every launch-kernel feature in one run — volumes (all kinds, PVCs through the listers, zones),
    SelectorSpread over services / RCs / RSs / StatefulSets, selectors, taints, host ports, extended
    resources, node conditions — 160 nodes × 1,500 pods against the object oracle."""
    from ksim import spread
    from workloads import rnd_mixed_workload
    monkeypatch.setenv("KUBE_MAX_PD_VOLS", "4")
    nodes, running, pods, pvs, pvcs, objs = rnd_mixed_workload(seed, n_nodes=160, n_pods=1500)
    preds = [k for k in scheduler.DEFAULT_PREDICATES if k != "MatchInterPodAffinity"]
    prios = [(n, w) for n, w in scheduler.DEFAULT_PRIORITIES if n != "InterPodAffinityPriority"]
    custom = {k: v for k, v in R.volume_predicates(R.VolumeListers(pvs, pvcs), 4).items() if k in preds}
    want, want_lni = R.simulate(nodes, running, pods, set(preds), list(prios), custom, spread=R.SpreadListers(**objs))
    cc = scheduler.ClusterCapacity(nodes, running, pods, predicates=preds, priorities=prios, pvs=pvs, pvcs=pvcs,
                                   spread=spread.SpreadListers(**objs))
    rep = cc.run()
    got = {n: (h, None) for n, h in rep.successful}
    got.update({n: (None, m) for n, m in rep.failed})
    assert [n for n, _ in rep.successful] == [n for n, h, _ in want if h is not None]
    for name, host, msg in want:
        assert got[name] == (host, msg), name
    assert rep.last_node_index == want_lni


@pytest.mark.parametrize("seed", [5, 12])
def test_cached_fast_form_matches_uncached_and_c_oracle(seed, monkeypatch):
    """The fast kernel's cached form (per (tree class, row) evaluations kept in LDS, only the
    committed row re-evaluated) and, with KSIM_NO_PCACHE, the uncached form over the same queue
    driven past saturation: identical placements, FitError histograms, counter and node state,
    both equal to the C oracle's (least_requested.go:36-53, balanced_resource_allocation.go:39-61,
    generic_scheduler.go:183-198)."""
    import cpu_ref
    from ksim import synth
    n, m = 9000, 60000
    r = synth.splitmix64(seed, 2 * n + 2 * m)
    cpu = synth._pick(r[0:n], [2000, 4000, 8000]) * 1
    mem = synth._pick(r[n:2 * n], [4 * synth.GI, 8 * synth.GI, 16 * synth.GI])
    pcpu = synth._pick(r[2 * n:2 * n + m], [100, 250, 500, 1000, 2000])
    pmem = synth._pick(r[2 * n + m:], [256 * synth.MI, 512 * synth.MI, synth.GI, 2 * synth.GI])
    names = ["c-%06d" % i for i in range(n)]
    preds = list(scheduler.DEFAULT_PREDICATES)
    prios = [("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]
    res = []
    for env in (None, "1"):
        if env:
            monkeypatch.setenv("KSIM_NO_PCACHE", env)
        cl = synth.resource_cluster(names, cpu, mem, np.full(n, 30, np.int32), pcpu, pmem)
        g = scheduler.GenericScheduler(cl, preds, prios, mode=abi.MODE_PERSISTENT)
        o1, r1, _ = g.schedule(0, 25000)
        o2, r2, _ = g.schedule(25000, m - 25000)
        res.append((np.concatenate([o1, o2]), np.concatenate([r1, r2]), g.last_node_index, g.node_state()))
        monkeypatch.delenv("KSIM_NO_PCACHE", raising=False)
    (o1, r1, c1, s1), (o2, r2, c2, s2) = res
    assert (o1 < 0).sum() > 1000 and (o1 >= 0).sum() > 1000  # saturated: FitErrors with reasons
    assert np.array_equal(o1, o2) and np.array_equal(r1, r2) and c1 == c2
    ref, ref_reasons, ref_state, ref_ctr = cpu_ref.run(cl, scheduler.make_config(preds, prios), threads=8)
    assert np.array_equal(o1, ref) and np.array_equal(r1, ref_reasons) and c1 == ref_ctr
    for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pod_count"):
        assert np.array_equal(s1[k], ref_state[k]), k
        assert np.array_equal(s2[k], ref_state[k]), k
