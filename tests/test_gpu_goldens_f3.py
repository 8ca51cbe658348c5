"""The reference's own test tables for inter-pod affinity and the Policy label priorities, through
the HIP kernels (the CPU oracle runs the same tables in test_oracle_interpod.py /
test_oracle_golden.py):

- TestInterPodAffinity / TestInterPodAffinityWithMultipleNodes (predicates_test.go:2168-3146): the
  verdict and failure reasons of MatchInterPodAffinity on every node, from ksim_evaluate;
- TestInterPodAffinityPriority / TestHardPodAffinitySymmetricWeight (interpod_affinity_test.go:42-615):
  the nodes selectHost picks for every lastNodeIndex over two periods equal the expected score
  vector's top nodes in descending name order;
- TestNewNodeLabelPriority (node_label_test.go:30-128) and TestZoneSpreadPriority without services
  selecting the pod (selector_spreading_test.go:605-760) the same way;
- TestServiceAffinity (predicates_test.go:1460-1620) cases where no service selects the pod.

The Go harnesses differ from the scheduler in what the predicate metadata sees (make_golden.py):
single node — every listed pod sits on the test node, the metadata sees the node's own pods;
multiple nodes — pods on their own nodes, the metadata sees the node under test's pods (or every
pod, "nometa").  A cluster is built per tested node that reproduces exactly that view: pods the
metadata does not see keep their labels (they still count for the incoming pod's terms) but lose
their required anti-affinity terms; the single-node harness's other pods sit on a twin of the test
node (same labels), which shares every topology domain except the node itself, as FakeNodeInfo's
pod lister does (hostname terms look at the node's own pods only, predicates.go:1176-1179)."""
import copy

import pytest

import ksim_ref as R
from golden_util import case_id, load
from ksim import abi, ingest, scheduler

pytestmark = pytest.mark.gpu


def _name(o):
    return (o.get("metadata") or {}).get("name", "")


def _node_name(p):
    return (p.get("spec") or {}).get("nodeName", "")


def _strip_anti(p):
    q = copy.deepcopy(p)
    a = (q.get("spec") or {}).get("affinity") or {}
    a.pop("podAntiAffinity", None)
    return q


def _evaluate(nodes, running, pod, preds, prios=(), **kw):
    """(fit, reason strings) per node name for one queued pod, without commit (ksim_evaluate)."""
    cl = ingest.Cluster.from_objects(nodes, running, [pod])
    g = scheduler.GenericScheduler(cl, preds, list(prios), mode=abi.MODE_LAUNCH, **kw)
    try:
        fit, rs, _, _ = g.evaluate(0)
    finally:
        g.close()
    return {nm: (bool(f), set(scheduler.reason_strings(int(m)))) for nm, f, m in zip(cl.names, fit, rs)}


def _oracle_errs(c, node):
    """The object oracle's error on this node (the reference returns an error, not a verdict)."""
    by_name = {_name(n): n for n in c["nodes"]}
    on_node = [p for p in c["pods"] if _node_name(p) == _name(node)]
    all_pods = [(p, node) for p in c["pods"]] if c["single_node"] else [(p, by_name[_node_name(p)]) for p in c["pods"]]
    node_pods = [(p, node) for p in on_node]
    try:
        meta = R.matching_anti_affinity_terms(c["pod"], all_pods if c["nometa"] else node_pods)
        _, _, err = R.interpod_affinity_matches(c["pod"], node, meta, all_pods, node_pods)
    except R.AffinityError as e:
        return e
    return err


@pytest.mark.parametrize("c", load("interpod_predicates"), ids=case_id)
def test_golden_interpod_predicate_on_gpu(c):
    for node in c["nodes"]:
        nm = _name(node)
        if c["single_node"]:
            twin = copy.deepcopy(node)
            twin["metadata"]["name"] = nm + "-twin"
            nodes = [node, twin]
            running = []
            for p in c["pods"]:
                q = copy.deepcopy(p) if _node_name(p) == nm else _strip_anti(p)
                q.setdefault("spec", {})["nodeName"] = nm if _node_name(p) == nm else nm + "-twin"
                running.append(q)
        else:
            nodes = c["nodes"]
            running = [p if (c["nometa"] or _node_name(p) == nm) else _strip_anti(p) for p in c["pods"]]
        for k, p in enumerate(running):
            p.setdefault("metadata", {}).setdefault("name", "golden-%d" % k)
        try:
            got = _evaluate(nodes, running, c["pod"], ["MatchInterPodAffinity"])
        except abi.KsimUnsupported:
            # refused up front exactly where the reference errs (e.g. an empty topologyKey)
            assert _oracle_errs(c, node) is not None, nm
            continue
        fits, reasons = got[nm]
        if not fits:
            assert reasons == set(c["reasons"][nm]), nm
        if (R._affinity(c["pod"]).get("nodeAffinity") is not None) and not c["single_node"]:
            sel = _evaluate(nodes, running, c["pod"], ["MatchNodeSelector"])
            fits = fits and sel[nm][0]   # the multi-node harness ANDs PodMatchNodeSelector
        assert fits == c["fits"][nm], nm


def _tied_top(expect):
    best = max(expect.values())
    return sorted((h for h, s in expect.items() if s == best), key=lambda h: h.encode(), reverse=True)


def _selects(nodes, running, pod, prios, expect, **kw):
    """selectHost over every lastNodeIndex of two periods lands on the expected top nodes from the
    highest name down (generic_scheduler.go:183-198)."""
    tied = _tied_top(expect)
    hard = kw.pop("hard_weight", 10)
    for k in range(2 * len(tied)):
        cl = ingest.Cluster.from_objects(nodes, running, [pod], hard_weight=hard)
        g = scheduler.GenericScheduler(cl, [], prios, mode=abi.MODE_AUTO, last_node_index=k, **kw)
        try:
            out, _, _ = g.schedule(0, 1)
        finally:
            g.close()
        assert cl.names[int(out[0])] == tied[k % len(tied)], (k, tied)


@pytest.mark.parametrize("c", load("interpod_priorities"), ids=case_id)
def test_golden_interpod_priority_selects_on_gpu(c):
    names = {_name(n) for n in c["nodes"]}
    # CreateNodeNameToInfoMap: pods of unknown nodes go to a node-less info the priority skips
    running = [p for p in c["pods"] if _node_name(p) in names]
    for k, p in enumerate(running):
        p.setdefault("metadata", {}).setdefault("name", "golden-%d" % k)
    _selects(c["nodes"], running, c["pod"], [("InterPodAffinityPriority", 1)], c["expect"], hard_weight=c["hard_weight"])


LABEL_CASES = [c for c in load("label_priorities") if c["kind"] == "labelPreference" or not c["services"]]


@pytest.mark.parametrize("c", LABEL_CASES, ids=case_id)
def test_golden_label_priorities_select_on_gpu(c):
    spec = ("labelPreference", c["label"], c["presence"]) if c["kind"] == "labelPreference" else \
        ("serviceAntiAffinity", c["label"])
    names = {_name(n) for n in c["nodes"]}
    running = [p for p in c["pods"] if _node_name(p) in names]
    for k, p in enumerate(running):
        p.setdefault("metadata", {}).setdefault("name", "golden-%d" % k)
    _selects(c["nodes"], running, c["pod"], [("P", 1)], c["expect"], custom_priorities={"P": spec})


SVC_CASES = [c for c in load("service_affinity") if not c["services"]]


@pytest.mark.parametrize("c", SVC_CASES, ids=case_id)
def test_golden_service_affinity_on_gpu(c):
    names = {_name(n) for n in c["nodes"]}
    running = [p for p in c["pods"] if _node_name(p) in names]
    got = _evaluate(c["nodes"], running, c["pod"], ["CheckServiceAffinity"], service_affinity=c["labels"])
    fits, reasons = got[_name(c["node"])]
    assert fits == c["fits"]
    if not fits:
        assert reasons == {"node(s) didn't match service affinity"}
