"""GPU parity of CheckServiceAffinity with services selecting the pods (predicates.go:920-1016; the
lender check of include/ksim.h ksim_affinity_tables.svc_*):

- the reference's TestServiceAffinity cases with services (predicates_test.go:1460-1620): the
  verdict on the node under test from ksim_evaluate, the case's pods cached on their nodes;
- random simulations against the object oracle reading the live scheduler cache as its pod lister
  (tests/test_oracle_c_features.py svc_simulate): identical placements, FitError texts and
  lastNodeIndex, and KSIM_E_UNSUPPORTED exactly where the oracle meets lenders that disagree on an
  open label (the reference's answer would depend on the pod lister's map order);
- in the launch form and the general persistent kernel;
- every per-pod form (ksim_schedule_one + assume, or the adapter's SCHEDULE_ONLY + ksim_pod_add)
  against the batch."""
import copy

import pytest

from golden_util import case_id, load
from ksim import abi, ingest, scheduler, spread
from test_oracle_c_features import SVC_PREDS, SVC_PRIOS, Ambiguous, svc_simulate
from workloads import rnd_svc_affinity_workload

pytestmark = pytest.mark.gpu


def _ns(o, names):
    """The golden JSON keeps Go identifiers as {"__ident__": ...}: one string per identifier."""
    o = copy.deepcopy(o)
    md = o.setdefault("metadata", {})
    ns = md.get("namespace")
    if isinstance(ns, dict):
        md["namespace"] = names.setdefault(ns.get("__ident__", ""), "ident-%d" % len(names))
    return o


SVC_CASES = [c for c in load("service_affinity") if c["services"]]


@pytest.mark.parametrize("c", SVC_CASES, ids=case_id)
def test_golden_service_affinity_with_services_on_gpu(c):
    names = {"metav1.NamespaceDefault": "default"}
    node_names = {(n.get("metadata") or {}).get("name", "") for n in c["nodes"]}
    running = [_ns(p, names) for p in c["pods"] if (p.get("spec") or {}).get("nodeName", "") in node_names]
    for k, p in enumerate(running):
        p["metadata"].setdefault("name", "golden-%d" % k)
    lst = spread.SpreadListers(services=[_ns(s, names) for s in c["services"]])
    cl = ingest.Cluster.from_objects(c["nodes"], running, [_ns(c["pod"], names)], spread=lst,
                                     service_affinity=c["labels"])
    g = scheduler.GenericScheduler(cl, ["CheckServiceAffinity"], [], mode=abi.MODE_LAUNCH, service_affinity=c["labels"])
    try:
        fit, rs, _, _ = g.evaluate(0)
    finally:
        g.close()
    k = cl.names.index(c["node"]["metadata"]["name"])
    assert bool(fit[k]) == c["fits"]
    if not c["fits"]:
        assert set(scheduler.reason_strings(int(rs[k]))) == {"node(s) didn't match service affinity"}


def _gpu_run(nodes, running, pods, services, aff_labels, mode=abi.MODE_AUTO):
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order, spread=spread.SpreadListers(services=services),
                                     service_affinity=aff_labels)
    g = scheduler.GenericScheduler(cl, SVC_PREDS, SVC_PRIOS, mode=mode, service_affinity=aff_labels)
    try:
        out, reasons, st = g.schedule()
        lni = g.last_node_index
    finally:
        g.close()
    res = [(cl.pod_names[k], cl.names[w] if w >= 0 else None,
            None if w >= 0 else scheduler.fit_error_message(cl.n_nodes, reasons[k], cl.scalar_names.items))
           for k, w in enumerate(out)]
    return res, lni, st


@pytest.mark.parametrize("mode", [abi.MODE_LAUNCH, abi.MODE_PERSISTENT])
@pytest.mark.parametrize("variant", ["consistent", "mixed_labels", "conflicting_running"])
@pytest.mark.parametrize("seed", range(4))
def test_service_affinity_simulation_matches_oracle(seed, variant, mode):
    """The launch form and the general persistent kernel (ksim_pgen.hip: the lender check over the
    row form and each workgroup's domain-0 copies of the totals)."""
    aff_labels = ["region", "rack"]
    nodes, running, pods, services = rnd_svc_affinity_workload(seed, mixed_labels=variant == "mixed_labels",
                                                               conflicting_running=variant == "conflicting_running",
                                                               full_labels=variant == "consistent")
    try:
        want, lni = svc_simulate(nodes, running, pods, SVC_PREDS, SVC_PRIOS, aff_labels, services)
    except Ambiguous:
        with pytest.raises(abi.KsimUnsupported):
            _gpu_run(nodes, running, pods, services, aff_labels, mode=mode)
        return
    got, ctr, st = _gpu_run(nodes, running, pods, services, aff_labels, mode=mode)
    assert st.mode == mode
    assert got == want
    assert ctr == lni


def test_schedule_one_with_service_affinity_matches_batch():
    """Pod by pod through ksim_schedule_one + assume (the scan kernel's commit records the lenders'
    disagreements like the batch's) == ksim_schedule."""
    import ctypes as C
    aff_labels = ["region", "rack"]
    nodes, running, pods, services = rnd_svc_affinity_workload(0, n_pods=80, full_labels=True)
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order, spread=spread.SpreadListers(services=services),
                                     service_affinity=aff_labels)
    batch = scheduler.GenericScheduler(cl, SVC_PREDS, SVC_PRIOS, mode=abi.MODE_LAUNCH, service_affinity=aff_labels)
    one = scheduler.GenericScheduler(cl, SVC_PREDS, SVC_PRIOS, mode=abi.MODE_LAUNCH, service_affinity=aff_labels)
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


PER_POD_FORMS = {
    "one_wg": {},                                            # <= 1,024 nodes: the single-workgroup kernel
    "resident": {"KSIM_ONE_WG": "0"},                        # the pick body in the resident kernel
    "scan": {"KSIM_ONE_WG": "0", "KSIM_NO_PICK": "1"},       # the multi-block scan
}


@pytest.mark.parametrize("pattern", ["assume", "adapter"])
@pytest.mark.parametrize("form", sorted(PER_POD_FORMS))
@pytest.mark.parametrize("variant", ["consistent", "mixed_labels", "conflicting_running"])
@pytest.mark.parametrize("seed", range(2))
def test_per_pod_forms_with_service_affinity_match_batch(seed, variant, form, pattern, monkeypatch, capfd):
    """Every per-pod form evaluates the lender check on the global counts the previous commit left
    (ksim_svc_lender) and records the lenders' disagreements at its commit (ksim_svc_commit):
    placements and lastNodeIndex == the batch's; KSIM_E_UNSUPPORTED exactly when the batch refuses.
    adapter: SCHEDULE_ONLY, then ksim_pod_add onto the chosen node (no tentative commit with these
    tables: a commit's recorded disagreements are not undone)."""
    import ctypes as C
    for k, v in PER_POD_FORMS[form].items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("KSIM_SERVE_STATS", "1")
    aff_labels = ["region", "rack"]
    nodes, running, pods, services = rnd_svc_affinity_workload(seed, n_pods=60, mixed_labels=variant == "mixed_labels",
                                                               conflicting_running=variant == "conflicting_running",
                                                               full_labels=variant == "consistent")
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order, spread=spread.SpreadListers(services=services),
                                     service_affinity=aff_labels)
    batch = scheduler.GenericScheduler(cl, SVC_PREDS, SVC_PRIOS, mode=abi.MODE_LAUNCH, service_affinity=aff_labels)
    one = scheduler.GenericScheduler(cl, SVC_PREDS, SVC_PRIOS, mode=abi.MODE_LAUNCH, service_affinity=aff_labels)
    ports, sc = cl.pod_ports, cl.pod_scalars
    try:
        try:
            out, _, _ = batch.schedule()
        except abi.KsimUnsupported:
            out = None
        refused = False
        for k in range(len(order)):
            pod = abi.Pod.from_buffer_copy(cl.pods[k].tobytes())
            res = abi.Result()
            try:
                one.h.call("ksim_schedule_one", C.byref(pod), abi.vptr(ports), len(ports), abi.vptr(sc), len(sc),
                           abi.SCHEDULE_ASSUME if pattern == "assume" else abi.SCHEDULE_ONLY, C.byref(res))
            except abi.KsimUnsupported:
                refused = True
                break
            if out is not None:
                assert res.node == out[k], k
            if pattern == "adapter" and res.node >= 0:
                one.h.call("ksim_pod_add", int(res.node), C.byref(pod), abi.vptr(ports), len(ports), abi.vptr(sc), len(sc))
        assert refused == (out is None)
        if out is not None:
            assert one.last_node_index == batch.last_node_index
        else:
            # the refusal is the call's: the handle goes on deciding (the next pod through any form)
            pod = abi.Pod.from_buffer_copy(cl.pods[0].tobytes())
            res = abi.Result()
            try:
                one.h.call("ksim_schedule_one", C.byref(pod), abi.vptr(ports), len(ports), abi.vptr(sc), len(sc),
                           abi.SCHEDULE_ONLY, C.byref(res))
            except abi.KsimUnsupported:
                pass
    finally:
        batch.close()
        one.close()
    # the form ran: the resident kernel took messages exactly in the resident form
    served = "[ksim serve]" in capfd.readouterr().err
    assert served == (form == "resident")


@pytest.mark.parametrize("variant", ["consistent", "mixed_labels", "conflicting_running"])
def test_service_affinity_at_scale_persistent_matches_launch(variant):
    """2,000 nodes (8 workgroups of the general persistent kernel: the lender's totals replicated in
    each, the disagreement bits released with the commit word) == the launch form, refusals
    included."""
    aff_labels = ["region", "rack"]
    nodes, running, pods, services = rnd_svc_affinity_workload(7, n_nodes=2000, n_pods=600,
                                                               mixed_labels=variant == "mixed_labels",
                                                               conflicting_running=variant == "conflicting_running",
                                                               full_labels=variant == "consistent")
    res = {}
    for mode in (abi.MODE_LAUNCH, abi.MODE_PERSISTENT):
        try:
            got, ctr, st = _gpu_run(nodes, running, pods, services, aff_labels, mode=mode)
            assert st.mode == mode
            res[mode] = (got, ctr)
        except abi.KsimUnsupported:
            res[mode] = "refused"
    assert res[abi.MODE_PERSISTENT] == res[abi.MODE_LAUNCH]
    if variant == "consistent":  # (lenders on one region / rack each, full labels: nothing to refuse)
        assert res[abi.MODE_LAUNCH] != "refused"
