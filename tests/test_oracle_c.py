"""The table-level C oracle (oracle/cpu_ref.c) pinned to the object-level restatement
(oracle/ksim_ref.py, itself pinned by the reference's golden vectors): same placements, bind
order, FitError messages and lastNodeIndex on seeded Kubernetes-shaped workloads (labels,
taints, conditions, host ports, selectors, node affinity, init containers, extended
resources, nodeName) and on a prefix of C2.  CPU only — this is what lets the GPU tests use
cpu_ref as the checker at sizes the Python oracle cannot reach."""
import pytest

import cpu_ref
import ksim_ref as R
from ksim import ingest, scheduler, synth
from workloads import add_prefer_avoid, rnd_workload

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


def c_oracle(nodes, running, pods, preds, prios, threads=2):
    """The simulator's loop on the C oracle: pods popped LIFO (store.go:223-233)."""
    cl = ingest.Cluster.from_objects(nodes, running, list(reversed(pods)))
    tables, na_add = scheduler.class_tables_for(cl.tables, prios)
    out, reasons, _, ctr = cpu_ref.run(cl, scheduler.make_config(preds, prios), threads=threads, tables=tables,
                                       na_add=na_add)
    res = []
    for k, w in enumerate(out):
        if w >= 0:
            res.append((cl.pod_names[k], cl.names[w], None))
        else:
            res.append((cl.pod_names[k], None,
                        scheduler.fit_error_message(cl.n_nodes, reasons[k], cl.scalar_names.items)))
    return res, ctr


@pytest.mark.parametrize("policy", sorted(POLICIES))
@pytest.mark.parametrize("seed", range(5))
def test_c_oracle_matches_object_oracle(seed, policy):
    nodes, running, pods = rnd_workload(100 + seed, n_nodes=19 + seed * 13, n_pods=160)
    preds, prios = POLICIES[policy]
    want, want_lni = R.simulate(nodes, running, pods, set(preds), list(prios))
    got, ctr = c_oracle(nodes, running, pods, preds, prios)
    assert got == want
    assert ctr == want_lni


PA_POLICIES = {
    "default": scheduler.provider("DefaultProvider"),
    "pa_only": (["GeneralPredicates"], [("NodePreferAvoidPodsPriority", 3)]),
    "pa_affinity": (["GeneralPredicates", "PodToleratesNodeTaints"],
                    [("NodePreferAvoidPodsPriority", 2), ("NodeAffinityPriority", 3), ("TaintTolerationPriority", 1),
                     ("LeastRequestedPriority", 1)]),
}


@pytest.mark.parametrize("policy", sorted(PA_POLICIES))
@pytest.mark.parametrize("seed", range(4))
def test_c_oracle_matches_object_oracle_prefer_avoid(seed, policy):
    """NodePreferAvoidPods with RC / RS-owned pods and preferAvoidPods annotations (case-varied
    field names, malformed JSON): the table-level oracle's per-class addends against the object
    oracle's CalculateNodePreferAvoidPodsPriorityMap."""
    nodes, running, pods = rnd_workload(300 + seed, n_nodes=21 + seed * 11, n_pods=140)
    nodes, pods = add_prefer_avoid(seed, nodes, pods)
    preds, prios = PA_POLICIES[policy]
    want, want_lni = R.simulate(nodes, running, pods, set(preds), list(prios))
    got, ctr = c_oracle(nodes, running, pods, preds, prios)
    assert got == want
    assert ctr == want_lni


def test_c_oracle_matches_object_oracle_on_c2_prefix():
    """C2's object shapes (selectors, host ports, NoSchedule / PreferNoSchedule taints,
    tolerations, BestEffort, NotReady / unschedulable nodes), scaled down so the cluster
    overflows."""
    nodes, pods = synth.c2_objects(25, 1200, seed=12)
    preds, prios = scheduler.provider("DefaultProvider")
    queue = list(reversed(pods))  # c2_objects returns scheduling order; the simulator pops LIFO
    want, want_lni = R.simulate(nodes, [], queue, set(preds), list(prios))
    got, ctr = c_oracle(nodes, [], queue, preds, prios)
    assert got == want
    assert ctr == want_lni
    assert sum(1 for _, h, _ in want if h is None) > 0  # the small cluster overflows: FitErrors covered
