"""GPU parity of the auxiliary counted priority (include/ksim.h ksim_affinity_tables.aux_*), the
second spreading priority a Policy can configure next to SelectorSpread:

- ServiceAntiAffinity with services selecting the pods (selector_spreading.go:180-275): the
  reference's TestZoneSpreadPriority cases with services (selector_spreading_test.go:605-760),
  checked by where selectHost puts the pod for every lastNodeIndex over two periods, and random
  simulations against the object oracle (placements, FitError texts, lastNodeIndex);
- ServiceSpreadingPriority configured together with SelectorSpreadPriority (the services-only
  selectors as the auxiliary pair, zones from utilnode.GetZoneKey), the same way.

Both launch forms (pass A fused into the scan, and as its own launch), the general persistent
kernel (ksim_pgen.hip: the auxiliary words of its pass-A record) and every per-pod form."""
import copy

import pytest

import ksim_ref as R
from golden_util import case_id, load
from ksim import abi, ingest, scheduler, spread
from workloads import rnd_spread_workload

pytestmark = pytest.mark.gpu

ZONE = "failure-domain.beta.kubernetes.io/zone"


def _ns_fix(o):
    """The golden JSON keeps Go identifiers as {"__ident__": ...}; NamespaceDefault is "default"."""
    o = copy.deepcopy(o)
    md = o.setdefault("metadata", {})
    if isinstance(md.get("namespace"), dict):
        md["namespace"] = "default"
    return o


SAA_CASES = [c for c in load("label_priorities") if c["kind"] == "serviceAntiAffinity" and c["services"]]


@pytest.mark.parametrize("c", SAA_CASES, ids=case_id)
def test_golden_service_anti_affinity_with_services_on_gpu(c):
    expect = c["expect"]
    best = max(expect.values())
    tied = sorted((h for h, s in expect.items() if s == best), key=lambda h: h.encode(), reverse=True)
    names = {(n.get("metadata") or {}).get("name", "") for n in c["nodes"]}
    running = [_ns_fix(p) for p in c["pods"] if (p.get("spec") or {}).get("nodeName", "") in names]
    for k, p in enumerate(running):
        p["metadata"].setdefault("name", "golden-%d" % k)
    pod = _ns_fix(c["pod"])
    lst = spread.SpreadListers(services=[_ns_fix(s) for s in c["services"]])
    for k in range(2 * len(tied)):
        cl = ingest.Cluster.from_objects(c["nodes"], running, [pod], spread=lst, aux=("service_anti_affinity", c["label"]))
        g = scheduler.GenericScheduler(cl, [], [("P", 1)], mode=abi.MODE_AUTO, last_node_index=k,
                                       custom_priorities={"P": ("serviceAntiAffinity", c["label"])})
        try:
            out, _, _ = g.schedule(0, 1)
        finally:
            g.close()
        assert cl.names[int(out[0])] == tied[k % len(tied)], (k, tied)


def _check(rep, want, want_lni):
    got = {name: (host, None) for name, host in rep.successful}
    got.update({name: (None, msg) for name, msg in rep.failed})
    assert [n for n, _ in rep.successful] == [n for n, h, _ in want if h is not None]
    for name, host, msg in want:
        assert got[name] == (host, msg), name
    assert rep.last_node_index == want_lni


def _saa_prios(seed):
    if seed % 2:
        return [("SAA", 3), ("SelectorSpreadPriority", 1), ("LeastRequestedPriority", 1)]
    return [("SAA", 2), ("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]


def _run(nodes, running, pods, preds, prios, lst, aux, custom=None, mode=abi.MODE_AUTO):
    """The simulator's loop (LIFO queue) through GenericScheduler on a cluster with `aux`, in `mode`
    (the launch form, or the general persistent kernel)."""
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order, spread=lst, aux=aux)
    assert cl.aux_active
    g = scheduler.GenericScheduler(cl, preds, prios, mode=mode, custom_priorities=custom)
    try:
        out, reasons, st = g.schedule()
        lni = g.last_node_index
    finally:
        g.close()
    assert st.mode == (abi.MODE_LAUNCH if mode == abi.MODE_LAUNCH else abi.MODE_PERSISTENT), st.mode
    rep = scheduler.Report()
    for k, w in enumerate(out):
        if w >= 0:
            rep.successful.append((cl.pod_names[k], cl.names[w]))
        else:
            rep.failed.append((cl.pod_names[k], scheduler.fit_error_message(cl.n_nodes, reasons[k], cl.scalar_names.items)))
    rep.last_node_index = lni
    return rep


@pytest.mark.parametrize("fuse", ["fused", "two_launch", "persistent"])
@pytest.mark.parametrize("seed", range(4))
def test_service_anti_affinity_simulation_matches_oracle(seed, fuse, monkeypatch):
    if fuse == "two_launch":
        monkeypatch.setenv("KSIM_FUSE_A", "0")
    mode = abi.MODE_PERSISTENT if fuse == "persistent" else abi.MODE_LAUNCH
    nodes, running, pods, objs = rnd_spread_workload(seed, zones=seed != 3)
    preds, _ = scheduler.provider("DefaultProvider")
    prios = _saa_prios(seed)
    want, want_lni = R.simulate(nodes, running, pods, set(preds), list(prios), spread=R.SpreadListers(**objs),
                                custom_priorities={"SAA": R.service_anti_affinity_priority(ZONE, R.SpreadListers(**objs))})
    rep = _run(nodes, running, pods, preds, prios, spread.SpreadListers(**objs), ("service_anti_affinity", ZONE),
               custom={"SAA": ("serviceAntiAffinity", ZONE)}, mode=mode)
    _check(rep, want, want_lni)


@pytest.mark.parametrize("fuse", ["fused", "two_launch", "persistent"])
@pytest.mark.parametrize("seed", range(4))
def test_both_spreading_priorities_match_oracle(seed, fuse, monkeypatch):
    """Through ClusterCapacity, which builds the cluster with the auxiliary pair itself."""
    if fuse == "two_launch":
        monkeypatch.setenv("KSIM_FUSE_A", "0")
    mode = abi.MODE_PERSISTENT if fuse == "persistent" else abi.MODE_LAUNCH
    nodes, running, pods, objs = rnd_spread_workload(seed, zones=seed != 3)
    preds = list(scheduler.DEFAULT_PREDICATES)
    prios = [("SelectorSpreadPriority", 1), ("ServiceSpreadingPriority", 2 + seed), ("LeastRequestedPriority", 1)]
    want, want_lni = R.simulate(nodes, running, pods, set(preds), list(prios), spread=R.SpreadListers(**objs))
    cc = scheduler.ClusterCapacity(nodes, running, pods, predicates=preds, priorities=prios,
                                   spread=spread.SpreadListers(**objs), mode=mode)
    assert cc.cluster.aux_active
    _check(cc.run(), want, want_lni)


def test_schedule_one_with_aux_matches_batch():
    """ksim_schedule_one (+ assume) pod by pod == ksim_schedule with the auxiliary priority (18
    nodes: the single-workgroup kernel, its pass A in LDS)."""
    import ctypes as C
    nodes, running, pods, objs = rnd_spread_workload(1, n_pods=60)
    order = list(reversed(pods))
    lst = spread.SpreadListers(**objs)
    cl = ingest.Cluster.from_objects(nodes, running, order, spread=lst, aux=("service_anti_affinity", ZONE))
    preds, _ = scheduler.provider("DefaultProvider")
    prios = _saa_prios(1)
    custom = {"SAA": ("serviceAntiAffinity", ZONE)}
    batch = scheduler.GenericScheduler(cl, preds, prios, mode=abi.MODE_LAUNCH, custom_priorities=custom)
    one = scheduler.GenericScheduler(cl, preds, prios, mode=abi.MODE_LAUNCH, custom_priorities=custom)
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


def test_aux_at_scale_matches_c_oracle():
    """2,000 nodes x 3,000 pods (8 blocks per pod, zone sums across blocks) against the C oracle, in
    the launch form and the general persistent kernel (several workgroups' domain sums: 40 rack
    domains; 80 exceed its pass-A record, and the persistent request runs in the launch form)."""
    import cpu_ref
    import random
    for racks in (40, 80):
        rng = random.Random(77)
        nodes, running, pods, objs = rnd_spread_workload(5, n_nodes=2000, n_pods=3000 if racks == 40 else 600,
                                                         n_running=400)
        for x in nodes:
            if rng.random() < 0.7:
                x["metadata"]["labels"]["rack"] = "r%d" % rng.randrange(racks)
        order = list(reversed(pods))
        lst = spread.SpreadListers(**objs)
        preds, _ = scheduler.provider("DefaultProvider")
        prios = [("SAA", 4), ("SelectorSpreadPriority", 1), ("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]
        custom = {"SAA": ("serviceAntiAffinity", "rack")}
        cl = ingest.Cluster.from_objects(nodes, running, order, spread=lst, aux=("service_anti_affinity", "rack"))
        p = scheduler.plan(cl, preds, prios, custom_priorities=custom)
        want, _, _, ctr, _ = cpu_ref.run(cl, None, threads=8, plan=p)
        for mode in (abi.MODE_LAUNCH, abi.MODE_PERSISTENT):
            g = scheduler.GenericScheduler(cl, preds, prios, custom_priorities=custom, mode=mode)
            try:
                out, _, st = g.schedule()
                assert st.mode == (abi.MODE_PERSISTENT if mode == abi.MODE_PERSISTENT and racks <= 64 else abi.MODE_LAUNCH)
                assert (out == want).all(), (racks, mode, int((out != want).argmax()))
                assert g.last_node_index == ctr
            finally:
                g.close()


PER_POD_FORMS = {
    "one_wg": {},                                            # <= 1,024 nodes: the single-workgroup kernel
    "resident": {"KSIM_ONE_WG": "0"},                        # the pick body in the resident kernel
    "scan": {"KSIM_ONE_WG": "0", "KSIM_NO_PICK": "1"},       # the multi-block scan with its pass A
}


def _aux_setup(kind, seed):
    """(workload, aux, prios, custom) of one auxiliary-priority family."""
    if kind == "saa_zone":
        return rnd_spread_workload(seed, n_pods=60), ("service_anti_affinity", ZONE), _saa_prios(seed), \
            {"SAA": ("serviceAntiAffinity", ZONE)}
    if kind == "saa_rack":  # 600 nodes (3 pick blocks), 40 rack domains next to the spread zones
        import random
        rng = random.Random(90 + seed)
        w = rnd_spread_workload(seed, n_nodes=600, n_pods=80, n_running=60)
        for x in w[0]:
            if rng.random() < 0.7:
                x["metadata"]["labels"]["rack"] = "r%d" % rng.randrange(40)
        prios = [("SAA", 4), ("SelectorSpreadPriority", 1), ("LeastRequestedPriority", 1)]
        return w, ("service_anti_affinity", "rack"), prios, {"SAA": ("serviceAntiAffinity", "rack")}
    prios = [("SelectorSpreadPriority", 1), ("ServiceSpreadingPriority", 2 + seed), ("LeastRequestedPriority", 1)]
    return rnd_spread_workload(seed, n_pods=60, zones=seed != 1), ("service_spreading",), prios, None


@pytest.mark.parametrize("pattern", ["assume", "adapter"])
@pytest.mark.parametrize("form", sorted(PER_POD_FORMS))
@pytest.mark.parametrize("kind", ["saa_zone", "saa_rack", "service_spreading"])
@pytest.mark.parametrize("seed", range(2))
def test_per_pod_forms_with_aux_match_batch(seed, kind, form, pattern, monkeypatch, capfd):
    """Every per-pod form reads the auxiliary priority: the single-workgroup kernel's pass A in LDS,
    the pick / resident kernels' pass-A record words (3 words and the domain sums after the spread
    zones), the scan's own pass A — placements and lastNodeIndex == the batch's.  adapter:
    SCHEDULE_ONLY (a tentative commit on the resident kernel), then ksim_pod_add onto the node."""
    import ctypes as C
    for k, v in PER_POD_FORMS[form].items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("KSIM_SERVE_STATS", "1")
    (nodes, running, pods, objs), aux, prios, custom = _aux_setup(kind, seed)
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order, spread=spread.SpreadListers(**objs), aux=aux)
    assert cl.aux_active
    preds, _ = scheduler.provider("DefaultProvider")
    batch = scheduler.GenericScheduler(cl, preds, prios, mode=abi.MODE_LAUNCH, custom_priorities=custom)
    one = scheduler.GenericScheduler(cl, preds, prios, mode=abi.MODE_LAUNCH, custom_priorities=custom)
    ports, sc = cl.pod_ports, cl.pod_scalars
    try:
        out, _, _ = batch.schedule()
        for k in range(len(order)):
            pod = abi.Pod.from_buffer_copy(cl.pods[k].tobytes())
            res = abi.Result()
            one.h.call("ksim_schedule_one", C.byref(pod), abi.vptr(ports), len(ports), abi.vptr(sc), len(sc),
                       abi.SCHEDULE_ASSUME if pattern == "assume" else abi.SCHEDULE_ONLY, C.byref(res))
            assert res.node == out[k], k
            if pattern == "adapter" and res.node >= 0:
                one.h.call("ksim_pod_add", int(res.node), C.byref(pod), abi.vptr(ports), len(ports), abi.vptr(sc), len(sc))
        assert one.last_node_index == batch.last_node_index
    finally:
        batch.close()
        one.close()
    # the form ran: the resident kernel took messages exactly in the resident form
    served = "[ksim serve]" in capfd.readouterr().err
    assert served == (form == "resident")


def _sharded_threads(cl, preds, prios, world, ranges, custom=None):
    """world node-sharded ranks of `cl` on this one device, driven from threads."""
    import threading
    import numpy as np
    scheds = [scheduler.ShardedScheduler(cl, preds, prios, r, world, custom_priorities=custom) for r in range(world)]
    scheduler.connect_local_world(scheds)
    outs = [[] for _ in range(world)]
    try:
        for first, count in ranges:
            errs = []

            def go(r):
                try:
                    outs[r].append(scheds[r].schedule(first, count)[0])
                except Exception as e:  # noqa: BLE001 — surfaced below
                    errs.append(e)
            ts = [threading.Thread(target=go, args=(r,)) for r in range(world)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            assert not errs, errs
        return scheduler.merge_sharded([np.concatenate(o) for o in outs]), [s.last_node_index for s in scheds]
    finally:
        for s in scheds:
            s.close()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("kind", ["saa_zone", "saa_rack", "service_spreading"])
def test_node_sharded_aux_matches_unsharded(kind, world, monkeypatch):
    """Node-sharded with the auxiliary priority (SURVEY.md §8e Phase A): its pair is node-keyed (each
    rank's own counts) and its key only groups the fit nodes' counts, so pass A exchanges its max /
    sum / haveZones and domain sums across the ranks after the spread zones.  Merged placements and
    every rank's lastNodeIndex == the unsharded launch form's (two calls: tags across calls)."""
    import numpy as np
    monkeypatch.setenv("KSIM_MAX_GRID", str(256 // world // 2))
    (nodes, running, pods, objs), aux, prios, custom = _aux_setup(kind, 1)
    if kind == "saa_rack":  # (<= 24 rack domains when sharded: SHARD_MAX_AUX_DOMAINS)
        for x in nodes:
            lab = x["metadata"]["labels"]
            if "rack" in lab:
                lab["rack"] = "r%d" % (int(lab["rack"][1:]) % 20)
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order, spread=spread.SpreadListers(**objs), aux=aux)
    preds, _ = scheduler.provider("DefaultProvider")
    g = scheduler.GenericScheduler(cl, preds, prios, mode=abi.MODE_LAUNCH, custom_priorities=custom)
    try:
        want, _, _ = g.schedule()
        want_ctr = g.last_node_index
    finally:
        g.close()
    half = len(order) // 2
    got, ctrs = _sharded_threads(cl, preds, prios, world, [(0, half), (half, len(order) - half)], custom)
    assert np.array_equal(got, want)
    assert ctrs == [want_ctr] * world


def test_node_sharded_aux_refuses_many_domains():
    """More auxiliary-priority domains than a sharded pass-A record holds: refused at the shard."""
    (nodes, running, pods, objs), aux, prios, custom = _aux_setup("saa_rack", 0)
    cl = ingest.Cluster.from_objects(nodes, running, list(reversed(pods)), spread=spread.SpreadListers(**objs), aux=aux)
    with pytest.raises(abi.KsimUnsupported):
        cl.shard(0, 300)
