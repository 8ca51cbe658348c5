"""The table-level C oracle (oracle/cpu_ref.c, the checker of every large GPU parity test) against
the object-level oracle (oracle/ksim_ref.py, pinned by the reference's golden vectors) at sizes
where ingest bugs would show: both are driven from the same Kubernetes-shaped objects, the C
oracle through ksim/ingest.py's interning (label sets, taint sets, host-port keys, pod classes,
reduce classes), the object oracle straight from the objects.  Placements, bind order, FitError
texts and lastNodeIndex must be identical, through high occupancy (1-fit shortcuts, ties, FitErrors).
CPU only."""
import pytest

import ksim_ref as R
from ksim import scheduler, synth
from test_oracle_c import c_oracle


def _check(nodes, queue, preds, prios, min_fail=0):
    want, want_lni = R.simulate(nodes, [], queue, set(preds), list(prios))
    got, ctr = c_oracle(nodes, [], queue, preds, prios, threads=8)
    assert len(got) == len(want)
    bad = [(w, g) for w, g in zip(want, got) if w != g]
    assert not bad, bad[:3]
    assert ctr == want_lni
    assert sum(1 for _, h, _ in want if h is None) >= min_fail
    return want


@pytest.mark.parametrize("n_nodes,n_pods,min_fail", [(400, 4000, 0), (120, 6000, 500)])
def test_c2_objects_at_scale(n_nodes, n_pods, min_fail):
    """C2-shaped objects (selectors, host ports, NoSchedule / PreferNoSchedule taints,
    tolerations, BestEffort, NotReady / unschedulable nodes): 400 nodes x 4,000 pods, and 120
    nodes x 6,000 pods, which drives the cluster past saturation (FitErrors for most late pods)."""
    nodes, pods = synth.c2_objects(n_nodes, n_pods, seed=31)
    preds, prios = scheduler.provider("DefaultProvider")
    want = _check(nodes, list(reversed(pods)), preds, prios, min_fail)  # c2_objects is in scheduling order
    assert len({h for _, h, _ in want if h}) > n_nodes // 2


def test_c1_objects_prefix():
    """C1 from objects (the README's node names, whose bytewise order differs from the numeric
    one, and etc/pod.yaml's pods): the B pods (cpu 100, never fit) then the first A pods."""
    nodes, expanded = synth.c1_objects()
    preds, prios = scheduler.provider("DefaultProvider")
    queue = expanded[-700:]  # the LIFO queue's first 700 pods: B x 10, then A
    want = _check(nodes, queue, preds, prios, min_fail=10)
    assert all(h is None for _, h, _ in want[:10]) and all(h for _, h, _ in want[10:])


def test_c1_objects_saturated_tail():
    """C1's end state: a scaled-down C1 (60 nodes, 32 pods each fit) filled past capacity, so
    the tail is all FitErrors ('Insufficient cpu'), the counter stops advancing and the
    1-fit shortcut is taken on the last free slots."""
    nodes, expanded = synth.c1_objects(n_nodes=60, n_a=60 * 32 + 25, n_b=3)
    preds, prios = scheduler.provider("DefaultProvider")
    want = _check(nodes, list(expanded), preds, prios, min_fail=28)
    assert sum(1 for _, h, _ in want if h) == 60 * 32
