"""The table-level C oracle (oracle/cpu_ref.c, ksim_ref_run_ex) over the inter-pod affinity,
SelectorSpread and volume tables, pinned to the object-level oracle (oracle/ksim_ref.py, itself
pinned by the reference's golden vectors: test_oracle_interpod.py, test_oracle_golden.py).  Both are
driven from the same Kubernetes-shaped objects — the C oracle through the product's ingest
(ksim/affinity.py, ksim/volumes.py, ksim/spread.py) and scheduler.plan, the object oracle straight
from the objects — so that GPU parity at C2x scale can use the C oracle without trusting the
ingest.  Placements, bind order, FitError texts and lastNodeIndex must be identical.  CPU only."""
import numpy as np
import pytest

import cpu_ref
import ksim_ref as R
from ksim import abi, ingest, scheduler, spread as ksp, synth
from workloads import (rnd_affinity_workload, rnd_mixed_workload, rnd_spread_workload, rnd_svc_affinity_workload,
                       rnd_volume_workload)

AFF_POLICIES = {
    "default": scheduler.provider("DefaultProvider"),
    "ipa_heavy": (list(scheduler.DEFAULT_PREDICATES), [("InterPodAffinityPriority", 7), ("LeastRequestedPriority", 1),
                                                       ("TaintTolerationPriority", 2)]),
    "predicate_only": (["MatchInterPodAffinity", "GeneralPredicates"], [("MostRequestedPriority", 1)]),
}


def c_oracle_objects(nodes, running, pods, preds, prios, pvs=(), pvcs=(), spread=None, threads=4,
                     spread_services_only=False, aux=None, custom_priorities=None, service_affinity=None):
    """The simulator's loop on the C oracle over the tables scheduler.plan builds: pods popped
    LIFO (store.go:223-233).  Returns ([(pod, node or None, FitError text or None)], lastNodeIndex)."""
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order, pvs=pvs, pvcs=pvcs, spread=spread,
                                     spread_services_only=spread_services_only, aux=aux, service_affinity=service_affinity)
    p = scheduler.plan(cl, preds, prios, custom_priorities=custom_priorities, service_affinity=service_affinity)
    out, reasons, _, ctr, _ = cpu_ref.run(cl, None, threads=threads, plan=p)
    res = []
    for k, w in enumerate(out):
        if w >= 0:
            res.append((cl.pod_names[k], cl.names[w], None))
        else:
            res.append((cl.pod_names[k], None, scheduler.fit_error_message(cl.n_nodes, reasons[k], cl.scalar_names.items)))
    return res, ctr


def _same(want, got):
    assert len(got) == len(want)
    bad = [(w, g) for w, g in zip(want, got) if w != g]
    assert not bad, bad[:3]


@pytest.mark.parametrize("policy", sorted(AFF_POLICIES))
@pytest.mark.parametrize("seed", range(4))
def test_affinity_matches_object_oracle(seed, policy):
    preds, prios = AFF_POLICIES[policy]
    nodes, running, pods = rnd_affinity_workload(seed, n_nodes=18 + 7 * seed, n_pods=90, n_running=12)
    want, lni = R.simulate(nodes, running, pods, set(preds), list(prios))
    got, ctr = c_oracle_objects(nodes, running, pods, preds, prios)
    _same(want, got)
    assert ctr == lni


@pytest.mark.parametrize("seed", range(4))
def test_volumes_match_object_oracle(seed, monkeypatch):
    monkeypatch.setenv("KUBE_MAX_PD_VOLS", "3")
    nodes, running, pods, pvs, pvcs = rnd_volume_workload(seed, zones=seed % 2 == 1, resolvable_only=seed % 2 == 1)
    preds = ["GeneralPredicates", "NoDiskConflict", "MaxEBSVolumeCount", "MaxGCEPDVolumeCount",
             "MaxAzureDiskVolumeCount"] + (["NoVolumeZoneConflict"] if seed % 2 else [])
    prios = [("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]
    custom = {k: v for k, v in R.volume_predicates(R.VolumeListers(pvs, pvcs), 3).items() if k in preds}
    want, lni = R.simulate(nodes, running, pods, set(preds), list(prios), custom)
    got, ctr = c_oracle_objects(nodes, running, pods, preds, prios, pvs=pvs, pvcs=pvcs)
    _same(want, got)
    assert ctr == lni
    assert any(m and ("disk" in m or "volume" in m) for _, _, m in want)   # the volume predicates decided something


@pytest.mark.parametrize("policy", ["default", "service"])
@pytest.mark.parametrize("seed", range(4))
def test_spread_matches_object_oracle(seed, policy):
    nodes, running, pods, objs = rnd_spread_workload(seed, zones=seed != 3)
    preds, prios = scheduler.provider("DefaultProvider")
    if policy == "service":
        prios = [("ServiceSpreadingPriority", 2), ("LeastRequestedPriority", 1)]
    want, lni = R.simulate(nodes, running, pods, set(preds), list(prios), spread=R.SpreadListers(**objs))
    got, ctr = c_oracle_objects(nodes, running, pods, preds, prios, spread=ksp.SpreadListers(**objs),
                                spread_services_only=policy == "service")
    _same(want, got)
    assert ctr == lni


ZONE = "failure-domain.beta.kubernetes.io/zone"


def _saa_prios(seed):
    if seed % 2:
        return [("SAA", 3), ("SelectorSpreadPriority", 1), ("LeastRequestedPriority", 1)]
    return [("SAA", 2), ("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]


@pytest.mark.parametrize("seed", range(4))
def test_service_anti_affinity_matches_object_oracle(seed):
    """A Policy's serviceAntiAffinity priority with services selecting the pods (the auxiliary
    counted priority, include/ksim.h ksim_affinity_tables.aux_*): the pods of the one selecting
    service counted per node and summed per zone-label value over the fit nodes
    (selector_spreading.go:180-275)."""
    nodes, running, pods, objs = rnd_spread_workload(seed, zones=seed != 3)
    preds, _ = scheduler.provider("DefaultProvider")
    prios = _saa_prios(seed)
    want, lni = R.simulate(nodes, running, pods, set(preds), list(prios), spread=R.SpreadListers(**objs),
                           custom_priorities={"SAA": R.service_anti_affinity_priority(ZONE, R.SpreadListers(**objs))})
    got, ctr = c_oracle_objects(nodes, running, pods, preds, prios, spread=ksp.SpreadListers(**objs),
                                aux=("service_anti_affinity", ZONE), custom_priorities={"SAA": ("serviceAntiAffinity", ZONE)})
    _same(want, got)
    assert ctr == lni


@pytest.mark.parametrize("seed", range(4))
def test_both_spreading_priorities_match_object_oracle(seed):
    """SelectorSpreadPriority and ServiceSpreadingPriority configured together with spread listers:
    the second one is the auxiliary counted priority over the services-only selectors."""
    nodes, running, pods, objs = rnd_spread_workload(seed, zones=seed != 3)
    preds, _ = scheduler.provider("DefaultProvider")
    prios = [("SelectorSpreadPriority", 1), ("ServiceSpreadingPriority", 2 + seed), ("LeastRequestedPriority", 1)]
    want, lni = R.simulate(nodes, running, pods, set(preds), list(prios), spread=R.SpreadListers(**objs))
    got, ctr = c_oracle_objects(nodes, running, pods, preds, prios, spread=ksp.SpreadListers(**objs),
                                aux=("service_spreading",))
    _same(want, got)
    assert ctr == lni


def test_service_anti_affinity_two_services_refused():
    """Two services selecting one pod: getFirstServiceSelector's pick is the lister's order."""
    nodes, running, pods, objs = rnd_spread_workload(0)
    objs["services"] = objs["services"] + [{"metadata": {"namespace": "ns1", "name": "dup"}, "spec": {"selector": {}}}]
    with pytest.raises(abi.KsimUnsupported):
        ingest.Cluster.from_objects(nodes, running, pods, spread=ksp.SpreadListers(**objs),
                                    aux=("service_anti_affinity", ZONE))


@pytest.mark.parametrize("seed", range(2))
def test_mixed_features_match_object_oracle(seed, monkeypatch):
    monkeypatch.setenv("KUBE_MAX_PD_VOLS", "4")
    nodes, running, pods, pvs, pvcs, objs = rnd_mixed_workload(seed, n_nodes=60, n_pods=500)
    preds = [k for k in scheduler.DEFAULT_PREDICATES if k != "MatchInterPodAffinity"]
    prios = [(n, w) for n, w in scheduler.DEFAULT_PRIORITIES if n != "InterPodAffinityPriority"]
    custom = {k: v for k, v in R.volume_predicates(R.VolumeListers(pvs, pvcs), 4).items() if k in preds}
    want, lni = R.simulate(nodes, running, pods, set(preds), list(prios), custom, spread=R.SpreadListers(**objs))
    got, ctr = c_oracle_objects(nodes, running, pods, preds, prios, pvs=pvs, pvcs=pvcs, spread=ksp.SpreadListers(**objs))
    _same(want, got)
    assert ctr == lni


def _c2x(n_nodes, n_pods, seed, threads):
    nodes, pods, pvs, pvcs, services = synth.c2x_objects(n_nodes, n_pods, seed)
    preds, prios = scheduler.provider("DefaultProvider")
    queue = list(reversed(pods))                    # c2x_objects is in scheduling order
    custom = {k: v for k, v in R.volume_predicates(R.VolumeListers(pvs, pvcs)).items() if k in preds}
    want, lni = R.simulate(nodes, [], queue, set(preds), list(prios), custom, spread=R.SpreadListers(services=services))
    got, ctr = c_oracle_objects(nodes, [], queue, preds, prios, pvs=pvs, pvcs=pvcs,
                                spread=ksp.SpreadListers(services=services), threads=threads)
    _same(want, got)
    assert ctr == lni
    return want


def test_c2x_objects_at_scale():
    """C2x (zones, GCE PD / EBS / zoned-PVC volumes, services → SelectorSpread, hostname
    anti-affinity) at 400 nodes x 4,000 pods, C oracle on 8 threads against the object oracle."""
    want = _c2x(400, 4000, 61, threads=8)
    assert len({h for _, h, _ in want if h}) > 300


def test_c2x_objects_saturated():
    """C2x scaled down until the cluster overflows: 40 nodes x 3,000 pods — FitErrors from
    resources, disk conflicts, volume counts and anti-affinity dominate the tail."""
    want = _c2x(40, 3000, 62, threads=3)
    fails = [m for _, h, m in want if h is None]
    assert len(fails) > 500


def _ns_default(o):
    """The golden JSON keeps Go identifiers as {"__ident__": ...}; NamespaceDefault is "default"."""
    import copy
    o = copy.deepcopy(o)
    md = o.setdefault("metadata", {})
    if isinstance(md.get("namespace"), dict):
        md["namespace"] = "default"
    return o


def test_golden_service_anti_affinity_with_services_c_oracle():
    """TestZoneSpreadPriority's cases with services (selector_spreading_test.go:605-760) through the
    product's ingest + scheduler.plan and the C oracle: selectHost over two periods of
    lastNodeIndex lands on the expected top nodes from the highest name down."""
    from golden_util import load
    cases = [c for c in load("label_priorities") if c["kind"] == "serviceAntiAffinity" and c["services"]]
    assert len(cases) == 7
    for c in cases:
        expect = c["expect"]
        best = max(expect.values())
        tied = sorted((h for h, s in expect.items() if s == best), key=lambda h: h.encode(), reverse=True)
        names = {(n.get("metadata") or {}).get("name", "") for n in c["nodes"]}
        running = [_ns_default(p) for p in c["pods"] if (p.get("spec") or {}).get("nodeName", "") in names]
        for k, p in enumerate(running):
            p["metadata"].setdefault("name", "golden-%d" % k)
        lst = ksp.SpreadListers(services=[_ns_default(s) for s in c["services"]])
        cl = ingest.Cluster.from_objects(c["nodes"], running, [_ns_default(c["pod"])], spread=lst,
                                         aux=("service_anti_affinity", c["label"]))
        p = scheduler.plan(cl, [], [("P", 1)], custom_priorities={"P": ("serviceAntiAffinity", c["label"])})
        for k in range(2 * len(tied)):
            out, _, _, _, _ = cpu_ref.run(cl, None, threads=1, plan=p, counter=k)
            assert cl.names[int(out[0])] == tied[k % len(tied)], (c["test"], k, tied)


class Ambiguous(Exception):
    """The object oracle met a pod whose service-affinity lenders disagree on an open label."""


def svc_simulate(nodes, running, pods, preds, prios, aff_labels, services):
    """The simulator's loop (LIFO) on the object oracle with CheckServiceAffinity reading the live
    scheduler cache as its pod lister (factory.go:166 podLister = schedulerCache): every cached pod,
    the running ones and those bound so far.  Raises Ambiguous where the pods a pod's labels select
    sit on nodes that disagree on a label its nodeSelector leaves open (filteredPods[0], a map order,
    would decide: predicates.go:1000-1008)."""
    infos = [R.NodeInfo(n) for n in nodes]
    by_name = {ni.name: ni for ni in infos}
    node_labels = {n["metadata"]["name"]: n["metadata"].get("labels") or {} for n in nodes}
    for q in running:
        if q["spec"].get("nodeName", "") in by_name:
            by_name[q["spec"]["nodeName"]].add_pod(q)

    def pred(pod, ni):
        cached = [q for x in infos for q in x.pods]
        md = pod.get("metadata") or {}
        ns, lab = md.get("namespace", ""), md.get("labels") or {}
        open_ = [l for l in aff_labels if l not in (pod["spec"].get("nodeSelector") or {})]
        svcs = [x for x in services if x["metadata"].get("namespace", "") == ns and x["spec"].get("selector") is not None
                and all(lab.get(k) == v for k, v in x["spec"]["selector"].items())]
        if open_ and svcs:
            lenders = {tuple(node_labels[q["spec"]["nodeName"]].get(l) for l in open_) for q in cached
                       if q["metadata"].get("namespace", "") == ns
                       and all((q["metadata"].get("labels") or {}).get(k) == v for k, v in lab.items())}
            if len(lenders) > 1:
                raise Ambiguous(md.get("name"))
        return R.new_service_affinity_predicate(aff_labels, services, cached, nodes)(pod, ni)

    sched = R.GenericScheduler(set(preds), list(prios), {"CheckServiceAffinity": pred})
    queue, out = list(pods), []
    while queue:
        pod = queue.pop()
        name = pod["metadata"]["name"]
        try:
            host = sched.schedule(pod, infos)
        except R.FitError as e:
            out.append((name, None, str(e)))
            continue
        bound = dict(pod, spec=dict(pod["spec"], nodeName=host))   # assume: Spec.NodeName = host (scheduler.go:366)
        by_name[host].add_pod(bound)
        out.append((name, host, None))
    return out, sched.last_node_index


SVC_PREDS = ["GeneralPredicates", "PodToleratesNodeTaints", "CheckServiceAffinity"]
SVC_PRIOS = [("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]


@pytest.mark.parametrize("variant", ["consistent", "mixed_labels", "conflicting_running"])
@pytest.mark.parametrize("seed", range(4))
def test_service_affinity_with_services_matches_object_oracle(seed, variant):
    """CheckServiceAffinity with services selecting the pods: the lender check over the counted
    pairs (include/ksim.h ksim_affinity_tables.svc_*) places like the object oracle reading the live
    cache, and refuses exactly where the oracle meets disagreeing lenders."""
    aff_labels = ["region", "rack"]
    nodes, running, pods, services = rnd_svc_affinity_workload(seed, mixed_labels=variant == "mixed_labels",
                                                               conflicting_running=variant == "conflicting_running",
                                                               full_labels=variant == "consistent")
    try:
        want, lni = svc_simulate(nodes, running, pods, SVC_PREDS, SVC_PRIOS, aff_labels, services)
    except Ambiguous:
        with pytest.raises(cpu_ref.Unsupported):
            c_oracle_objects(nodes, running, pods, SVC_PREDS, SVC_PRIOS, spread=ksp.SpreadListers(services=services),
                             service_affinity=aff_labels)
        return
    got, ctr = c_oracle_objects(nodes, running, pods, SVC_PREDS, SVC_PRIOS, spread=ksp.SpreadListers(services=services),
                                service_affinity=aff_labels)
    _same(want, got)
    assert ctr == lni
    if variant == "consistent":
        assert any(m and "service affinity" in m for _, _, m in want)   # the lenders constrained something


def wide_workload(seed, n_nodes=60, n_pods=300):
    """Taints, node selectors / affinity and preferAvoidPods with owned pods keeping their preferred
    node-affinity terms: pod classes with more than 16 (TaintToleration x NodeAffinity /
    NodePreferAvoidPods) reduce classes — the launch form's wide decision."""
    from workloads import add_prefer_avoid, rnd_workload
    nodes, running, pods = rnd_workload(seed, n_nodes=n_nodes, n_pods=n_pods)
    nodes, pods = add_prefer_avoid(seed, nodes, pods, keep_preferred=True)
    return nodes, running, pods


def very_wide_workload(seed, n_nodes=80, n_pods=300):
    """More than 16 values in ONE reduce dimension (formerly refused): nodes carry a `w` label out of
    40 values and 0..24 PreferNoSchedule taints; many pods prefer `w` values through six weighted
    terms (weights 1..32: up to 64 distinct preferred-weight sums over the label sets) and tolerate
    some of the taints (up to 25 distinct intolerable counts).  NormalizeReduce has no limit on the
    values (priorities/reduce.go:29-64)."""
    import random
    from workloads import rnd_workload
    rng = random.Random(seed * 104729 + 7)
    nodes, running, pods = rnd_workload(seed, n_nodes=n_nodes, n_pods=n_pods)
    for x in nodes:
        x["metadata"].setdefault("labels", {})["w"] = str(rng.randrange(40))
        k = rng.randrange(25)
        x["spec"]["taints"] = [t for t in x["spec"].get("taints") or [] if t["effect"] != "PreferNoSchedule"] + \
            [{"key": "pns-%d" % j, "value": "", "effect": "PreferNoSchedule"} for j in range(k)]
    for p in pods:
        spec = p["spec"]
        # (a pod's TaintToleration x NodeAffinity classes stay <= 256, the wide decision's bound:
        # the pods with many preferred-weight sums tolerate every PreferNoSchedule taint)
        if rng.random() < 0.5:
            terms = [{"weight": 1 << t, "preference": {"matchExpressions": [
                {"key": "w", "operator": "In", "values": [str(v) for v in rng.sample(range(40), 20)]}]}} for t in range(6)]
            spec.setdefault("affinity", {}).setdefault("nodeAffinity", {})[
                "preferredDuringSchedulingIgnoredDuringExecution"] = terms
            spec.setdefault("tolerations", []).append({"operator": "Exists", "effect": "PreferNoSchedule"})
        elif rng.random() < 0.5:
            spec.setdefault("tolerations", []).extend(
                {"key": "pns-%d" % j, "operator": "Exists", "effect": "PreferNoSchedule"} for j in rng.sample(range(25), 6))
    return nodes, running, pods


@pytest.mark.parametrize("seed", range(3))
def test_very_wide_reduce_dimension_matches_object_oracle(seed):
    """More than 16 values in one reduce dimension: ingest (value rows wider than 16, ABI 7) + plan +
    the C oracle against the object oracle."""
    nodes, running, pods = very_wide_workload(seed)
    preds, prios = scheduler.provider("DefaultProvider")
    want, lni = R.simulate(nodes, running, pods, set(preds), list(prios))
    got, ctr = c_oracle_objects(nodes, running, pods, preds, prios)
    _same(want, got)
    assert ctr == lni
    cl = ingest.Cluster.from_objects(nodes, running, list(reversed(pods)))
    t = scheduler.plan(cl, preds, prios).tables
    dims = np.maximum(np.asarray(t["n_tt"]), np.asarray(t["n_na"]))[np.asarray(cl.pods["cls"])]
    assert (dims > 16).any() and t["tt_val"].shape[1] > 16


@pytest.mark.parametrize("seed", range(4))
def test_wide_reduce_classes_match_object_oracle(seed):
    """More than 16 reduce classes per pod class (formerly refused): ingest + plan + the C oracle
    against the object oracle."""
    nodes, running, pods = wide_workload(seed)
    preds, prios = scheduler.provider("DefaultProvider")
    want, lni = R.simulate(nodes, running, pods, set(preds), list(prios))
    got, ctr = c_oracle_objects(nodes, running, pods, preds, prios)
    _same(want, got)
    assert ctr == lni
    cl = ingest.Cluster.from_objects(nodes, running, list(reversed(pods)))
    t = scheduler.plan(cl, preds, prios).tables
    k = (np.asarray(t["n_tt"]) * np.asarray(t["n_na"]))[np.asarray(cl.pods["cls"])]
    assert (k > 16).any()
