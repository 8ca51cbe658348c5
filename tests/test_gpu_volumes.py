"""GPU parity of the volume predicates (NoDiskConflict, MaxEBS / GCEPD / AzureDiskVolumeCount,
NoVolumeZoneConflict) through libksim.so's launch-mode kernels: the reference's own test tables
(predicates_test.go:669-891, 1622-2039, 3694-3913) evaluated on the device, and random simulations
against the object oracle (oracle/ksim_ref.py) — placements in bind order, FitError texts,
lastNodeIndex and the device's per-node volume mounts after the run."""
import numpy as np
import pytest

import ksim_ref as R
import volume_model as M
from golden_util import case_id, load
from ksim import abi, ingest, scheduler
from workloads import rnd_volume_workload

pytestmark = pytest.mark.gpu

VOLUME_KEYS = ["NoDiskConflict", "MaxEBSVolumeCount", "MaxGCEPDVolumeCount", "MaxAzureDiskVolumeCount"]


@pytest.mark.parametrize("c", load("volumes"), ids=case_id)
def test_golden_volume_predicates_on_gpu(c):
    mv = c["max_vols"]
    cl = ingest.Cluster.from_objects([c["node"]], c["pods"], [c["pod"]], pvs=c["pvs"], pvcs=c["pvcs"],
                                     max_vols=None if mv is None else (mv, mv, mv))
    g = scheduler.GenericScheduler(cl, [c["predicate"]], [("EqualPriority", 1)])
    fit, rs, _, _ = g.evaluate(0)
    assert bool(fit[0]) == c["fits"]
    if not c["fits"]:
        assert scheduler.reason_strings(int(rs[0])) == c["reasons"]
    g.close()


POLICIES = {
    # the volume predicates inside the default ordering, without CheckVolumeBinding (it errs on
    # every PVC the simulator's empty listers hold)
    "volumes_lr_bra": (["GeneralPredicates", "PodToleratesNodeTaints"] + VOLUME_KEYS,
                       [("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]),
    "volumes_only": (VOLUME_KEYS, [("MostRequestedPriority", 2)]),
}


def _run_both(nodes, running, pods, pvs, pvcs, preds, prios, mode, max_vols, chunks=None):
    listers = R.VolumeListers(pvs, pvcs)
    custom = {k: v for k, v in R.volume_predicates(listers, max_vols).items() if k in preds}
    want, want_lni = R.simulate(nodes, running, pods, set(preds), list(prios), custom_predicates=custom)
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order, pvs=pvs, pvcs=pvcs,
                                     max_vols=None if max_vols is None else (max_vols,) * 3)
    g = scheduler.GenericScheduler(cl, preds, prios, mode=mode)
    outs, hists = [], []
    for first, count in chunks or [(0, len(order))]:
        o, h, _ = g.schedule(first, count)
        outs.append(o)
        hists.append(h)
    out, hist = np.concatenate(outs), np.concatenate(hists)
    for k, (name, host, msg) in enumerate(want):
        assert cl.pod_names[k] == name
        w = int(out[k])
        if host is None:
            assert w == -1, (k, name)
            assert scheduler.fit_error_message(cl.n_nodes, hist[k], cl.scalar_names.items) == msg, name
        else:
            assert w >= 0 and cl.names[w] == host, (k, name, host)
    assert g.last_node_index == want_lni
    return cl, g, want


def _expected_mounts(cl, running, want, pods_by_name):
    mounts = [M.slots_of(cl.volumes, i) for i in range(cl.n_nodes)]  # the running pods' (loaded) state
    for k, (name, host, _) in enumerate(want):
        vc = int(cl.pods["vol_class"][k])
        if host is not None and vc:
            M.commit(mounts[cl.index[host]], cl.volumes, vc)
    return mounts


def _device_mounts(g, n):
    slots, cnt = g.volume_state()
    out = []
    for i in range(n):
        m = {}
        for s in range(int(cnt[i])):
            w = int(slots[s, i])
            m[w >> 32] = [w & 0x7FF, (w >> 11) & 0x7FF, (w >> 22) & 0x3FF]
        out.append(m)
    return out


@pytest.mark.parametrize("mode", [abi.MODE_LAUNCH, abi.MODE_AUTO])
@pytest.mark.parametrize("policy", sorted(POLICIES))
@pytest.mark.parametrize("seed", range(4))
def test_volume_simulation_matches_oracle(seed, policy, mode):
    nodes, running, pods, pvs, pvcs = rnd_volume_workload(seed)
    preds, prios = POLICIES[policy]
    max_vols = [None, 3, 2, 4][seed]
    cl, g, want = _run_both(nodes, running, pods, pvs, pvcs, preds, prios, mode, max_vols)
    assert _device_mounts(g, cl.n_nodes) == _expected_mounts(cl, running, want, None)
    g.close()


@pytest.mark.parametrize("seed", range(3))
def test_volume_zone_simulation_matches_oracle(seed):
    """NoVolumeZoneConflict on zone-labelled nodes with every PVC resolvable (the reference errs on
    the others), inside the default predicate set minus CheckVolumeBinding."""
    nodes, running, pods, pvs, pvcs = rnd_volume_workload(seed, zones=True, resolvable_only=True)
    preds = [k for k in scheduler.DEFAULT_PREDICATES if k not in ("CheckVolumeBinding", "MatchInterPodAffinity")]
    prios = [(n, w) for n, w in scheduler.DEFAULT_PRIORITIES if n != "InterPodAffinityPriority"]
    cl, g, want = _run_both(nodes, running, pods, pvs, pvcs, preds, prios, abi.MODE_AUTO, 3)
    g.close()


def test_volume_pods_between_resource_only_runs():
    """Ranges without volume pods take the persistent kernels (which never touch the volume
    slots); ranges with them the launch kernels — the state must carry across."""
    nodes, running, pods, pvs, pvcs = rnd_volume_workload(7, n_pods=150, p_vol=0.25)
    chunks = [(0, 7), (7, 1), (8, 40), (48, 2), (50, 100)]
    cl, g, want = _run_both(nodes, running, pods, pvs, pvcs, POLICIES["volumes_lr_bra"][0],
                            POLICIES["volumes_lr_bra"][1], abi.MODE_AUTO, 3, chunks)
    assert _device_mounts(g, cl.n_nodes) == _expected_mounts(cl, running, want, None)
    g.close()


def test_volume_release_restores_state():
    """ksim_assume then NodeInfo.RemovePod (ksim_pod_remove) of a volume pod: mounts return."""
    nodes, running, pods, pvs, pvcs = rnd_volume_workload(3, n_pods=30)
    cl = ingest.Cluster.from_objects(nodes, running, pods, pvs=pvs, pvcs=pvcs)
    g = scheduler.GenericScheduler(cl, VOLUME_KEYS, [("LeastRequestedPriority", 1)], mode=abi.MODE_LAUNCH)
    before = _device_mounts(g, cl.n_nodes)
    k = next(i for i in range(len(pods)) if cl.pods["vol_class"][i])
    node = 2
    g.h.call("ksim_assume", k, node)
    mid = _device_mounts(g, cl.n_nodes)
    assert mid != before
    p = np.ascontiguousarray(cl.pods[k:k + 1])
    g.h.call("ksim_pod_remove", node, abi.vptr(p), abi.vptr(cl.pod_ports), len(cl.pod_ports),
             abi.vptr(cl.pod_scalars), len(cl.pod_scalars))
    assert _device_mounts(g, cl.n_nodes) == before
    g.close()


def test_schedule_one_with_volumes_matches_batch():
    """ksim_schedule_one (+ assume) pod by pod == ksim_schedule on another handle: the per-pod
    entry point evaluates and commits volume pods through the same tables.  Five nodes with one
    volume of each MaxPD kind allowed: about half the queue fails, so FitError histograms are
    compared too."""
    import ctypes as C
    nodes, running, pods, pvs, pvcs = rnd_volume_workload(5, n_nodes=5, n_pods=60)
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order, pvs=pvs, pvcs=pvcs, max_vols=(1, 1, 1))
    preds, prios = POLICIES["volumes_lr_bra"]
    batch = scheduler.GenericScheduler(cl, preds, prios, mode=abi.MODE_LAUNCH)
    one = scheduler.GenericScheduler(cl, preds, prios, mode=abi.MODE_LAUNCH)
    try:
        out, reasons, _ = batch.schedule()
        assert (out < 0).sum() >= 10 and (out >= 0).sum() >= 10   # both outcomes exercised
        for k in range(len(order)):
            pod = abi.Pod.from_buffer_copy(cl.pods[k].tobytes())
            res = abi.Result()
            one.h.call("ksim_schedule_one", C.byref(pod), abi.vptr(cl.pod_ports), len(cl.pod_ports),
                       abi.vptr(cl.pod_scalars), len(cl.pod_scalars), abi.SCHEDULE_ASSUME, C.byref(res))
            assert res.node == out[k], k
            if res.node < 0:
                assert list(res.reasons) == list(reasons[k]), k
        assert one.last_node_index == batch.last_node_index
        assert _device_mounts(one, cl.n_nodes) == _device_mounts(batch, cl.n_nodes)
    finally:
        batch.close()
        one.close()
