"""Policy files → key sets (the simulator's Policy path, pkg/scheduler/simulator.go:382-421;
factory.CreateFromConfig, factory/factory.go:932-1001), pinned by the reference's own goldens:
algorithmprovider/defaults/compatibility_test.go (decoding of the 1.0 / 1.1 / 1.9 policies) and
api/validation/validation_test.go (ValidatePolicy's errors).  CPU only."""
import pytest

from golden_util import case_id, load
from ksim import abi, ingest, policy, scheduler


@pytest.mark.parametrize("c", load("policy"), ids=case_id)
def test_policy_decoding_golden(c):
    p = policy.decode(c["json"])
    assert [[n, a] for n, a in p.predicates] == c["predicates"]
    assert [[n, w, a] for n, w, a in p.priorities] == c["priorities"]


@pytest.mark.parametrize("c", load("policy_validation"), ids=case_id)
def test_policy_validation_golden(c):
    p = policy.decode(dict(c["policy"], kind="Policy"))
    if c["error"] is None:
        policy.validate(p)
    else:
        with pytest.raises(policy.PolicyError) as ei:
            policy.validate(p)
        assert str(ei.value) == c["error"]


def test_policy_errors_are_aggregated():
    p = policy.decode({"priorities": [{"name": "A", "weight": 0}, {"name": "B", "weight": -1}]})
    with pytest.raises(policy.PolicyError) as ei:
        policy.validate(p)
    assert str(ei.value) == ("[Priority A should have a positive weight applied to it or it has overflown, "
                             "Priority B should have a positive weight applied to it or it has overflown]")


def test_1_9_policy_key_sets():
    """The 1.9 compatibility policy: every built-in key runs (the custom-named TestServiceAffinity /
    TestLabelsPresence are registered but outside predicatesOrdering, so never evaluated)."""
    (c,) = [c for c in load("policy") if c["version"] == "1.9"]
    preds, prios, lp = policy.key_sets(policy.decode(c["json"]))
    assert lp is None
    assert "TestServiceAffinity" not in preds and "GeneralPredicates" in preds
    cfg = scheduler.make_config(preds, prios)
    assert cfg.weights[abi.W_LEAST] == 2 and cfg.weights[abi.W_MOST] == 2 and cfg.weights[abi.W_BALANCED] == 2
    assert cfg.weights[abi.W_TAINT_TOL] == 2 and cfg.weights[abi.W_NODE_AFF] == 2
    # EqualPriority 1 + ImageLocality 0 + SelectorSpread 10 + NodePreferAvoid 10 + InterPodAffinity 0, x 2
    assert cfg.const_score == 2 * (1 + 0 + 10 + 10 + 0)


def test_1_0_policy_custom_priorities():
    """The 1.0 compatibility policy's serviceAntiAffinity / labelPreference priorities register under
    their policy names (factory/plugins.go:271-323)."""
    (c,) = [c for c in load("policy") if c["version"] == "1.0"]
    pol = policy.decode(c["json"])
    _, prios, _ = policy.key_sets(pol)
    args = policy.priority_arguments(pol)
    assert args == {"TestServiceAntiAffinity": ("serviceAntiAffinity", "zone"),
                    "TestLabelPreference": ("labelPreference", "bar", True)}
    assert ("TestServiceAntiAffinity", 3) in prios and ("TestLabelPreference", 4) in prios
    with pytest.raises(abi.KsimUnsupported):
        policy.key_sets(policy.decode({"priorities": [{"name": "X", "weight": 1, "argument": {"bogus": {}}}]}))


def test_label_set_priorities_as_addends():
    """NodeLabel / ServiceAntiAffinity (no services) scores are functions of the label set: carried
    as per-NodeAffinity-class addends."""
    import ksim_ref as R
    from ksim import ingest
    nodes = [{"metadata": {"name": "n%d" % i, "labels": lab}, "status": {"allocatable": {"cpu": "1", "pods": "9"}}}
             for i, lab in enumerate([{}, {"bar": "1"}, {"zone": "a"}, {"bar": "2", "zone": "b"}])]
    cl = ingest.Cluster.from_objects(nodes, [], [{"metadata": {"name": "p"}, "spec": {}}])
    custom = {"LP": ("labelPreference", "bar", True), "SAA": ("serviceAntiAffinity", "zone")}
    t, add = scheduler.class_tables_for(cl.tables, [("LP", 4), ("SAA", 3)], cl.label_sets.items, custom)
    got = [int(add[0][t["na_class"][0][int(cl.cols["label_set"][i])]]) for i in range(4)]
    infos = [R.NodeInfo(x) for x in sorted(nodes, key=lambda x: x["metadata"]["name"].encode())]
    want = R.prioritize_nodes({"metadata": {}}, infos, [("LP", 4), ("SAA", 3)],
                              custom={"LP": R.node_label_priority("bar", True),
                                      "SAA": R.service_anti_affinity_priority("zone")})
    assert got == want


def test_missing_sections_use_default_provider_and_mandatory_predicate():
    preds, prios, _ = policy.key_sets(policy.decode({"kind": "Policy"}))
    d_preds, d_prios = scheduler.provider("DefaultProvider")
    assert sorted(preds) == sorted(d_preds) and prios == d_prios
    preds, prios, _ = policy.key_sets(policy.decode({"predicates": [{"name": "PodFitsResources"}],
                                                      "priorities": [{"name": "MostRequestedPriority", "weight": 3}]}))
    assert "CheckNodeCondition" in preds  # plugins.go:401-406 mandatory predicate
    assert scheduler.make_config(["PodFitsResources"], []).predicates & abi.P_CHECK_NODE_CONDITION


def test_label_presence_predicate_and_flags():
    preds, _, lp = policy.key_sets(policy.decode({"predicates": [
        {"name": "CheckNodeLabelPresence", "argument": {"labelsPresence": {"labels": ["retiring"], "presence": False}}}],
        "priorities": [{"name": "LeastRequestedPriority", "weight": 1}]}))
    assert lp == (["retiring"], False) and "CheckNodeLabelPresence" in preds
    fl = scheduler.label_presence_flags([{}, {"retiring": "2026"}, {"zone": "a"}], [0, 1, 2, 1], lp)
    assert list(fl) == [0, abi.N_LABEL_PRESENCE, 0, abi.N_LABEL_PRESENCE]
    assert scheduler.make_config(preds, []).predicates & abi.P_LABEL_PRESENCE


def test_extenders_and_always_check_all_unsupported():
    with pytest.raises(abi.KsimUnsupported):
        policy.key_sets(policy.decode({"extenders": [{"urlPrefix": "http://x", "filterVerb": "filter"}]}))
    with pytest.raises(abi.KsimUnsupported):
        policy.key_sets(policy.decode({"alwaysCheckAllPredicates": True}))


# ----------------------------------------------------------------------------- GPU: policy runs
GPU_POLICIES = {
    "absent_rank": {"predicates": [{"name": "GeneralPredicates"}, {"name": "PodToleratesNodeTaints"},
                                   {"name": "CheckNodeLabelPresence",
                                    "argument": {"labelsPresence": {"labels": ["rank"], "presence": False}}}],
                    "priorities": [{"name": "LeastRequestedPriority", "weight": 1},
                                   {"name": "ImageLocalityPriority", "weight": 2}]},
    "present_tier_disk": {"predicates": [{"name": "PodFitsResources"}, {"name": "MatchNodeSelector"},
                                         {"name": "CheckNodeLabelPresence",
                                          "argument": {"labelsPresence": {"labels": ["tier", "disk"], "presence": True}}}],
                          "priorities": [{"name": "MostRequestedPriority", "weight": 3},
                                         {"name": "BalancedResourceAllocation", "weight": 1},
                                         {"name": "EqualPriority", "weight": 1}]},
    "defaults_1_9_like": {"kind": "Policy"},
    "service_affinity": {"predicates": [{"name": "PodFitsResources"}, {"name": "PodToleratesNodeTaints"},
                                        {"name": "CheckServiceAffinity",
                                         "argument": {"serviceAffinity": {"labels": ["tier", "disk"]}}}],
                         "priorities": [{"name": "BalancedResourceAllocation", "weight": 1},
                                        {"name": "NodeAffinityPriority", "weight": 2}]},
    "label_priorities": {"predicates": [{"name": "GeneralPredicates"}, {"name": "PodToleratesNodeTaints"}],
                         "priorities": [{"name": "LeastRequestedPriority", "weight": 1},
                                        {"name": "PreferSsd", "weight": 3,
                                         "argument": {"labelPreference": {"label": "rank", "presence": True}}},
                                        {"name": "SpreadByTier", "weight": 2,
                                         "argument": {"serviceAntiAffinity": {"label": "tier"}}},
                                        {"name": "NodePreferAvoidPodsPriority", "weight": 10000}]},
}


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [abi.MODE_LAUNCH, abi.MODE_AUTO, abi.MODE_TREE])
@pytest.mark.parametrize("name", sorted(GPU_POLICIES))
def test_gpu_policy_run_matches_oracle(name, mode):
    """A Policy file through ClusterCapacity(policy_obj=...) vs the oracle run with the same key
    sets and the CheckNodeLabelPresence closure (predicates.go:875-910)."""
    import ksim_ref as R
    from workloads import rnd_workload
    pol = policy.decode(GPU_POLICIES[name])
    preds, prios, lp = policy.key_sets(pol)
    custom = {"CheckNodeLabelPresence": R.new_node_label_predicate(*lp)} if lp else {}
    if policy.service_affinity_labels(pol) is not None:
        custom["CheckServiceAffinity"] = R.new_service_affinity_predicate(policy.service_affinity_labels(pol))
    cprios = {n: (R.node_label_priority(a[1], a[2]) if a[0] == "labelPreference" else R.service_anti_affinity_priority(a[1]))
              for n, a in policy.priority_arguments(pol).items()}
    for seed in (3, 11):
        nodes, running, pods = rnd_workload(seed, n_nodes=31 + seed, n_pods=140)
        want, lni = R.simulate(nodes, running, pods, set(preds), list(prios), custom, custom_priorities=cprios)
        rep = scheduler.ClusterCapacity(nodes, running, pods, policy_obj=pol, mode=mode).run()
        got = {n: (h, None) for n, h in rep.successful}
        got.update({n: (None, m) for n, m in rep.failed})
        assert [n for n, _ in rep.successful] == [n for n, h, _ in want if h is not None]
        for pod, host, msg in want:
            assert got[pod] == (host, msg), pod
        assert rep.last_node_index == lni
        if lp and not lp[1]:
            assert any("didn't have the requested labels" in (m or "") for _, _, m in want)


def test_service_affinity_table_matches_oracle():
    """CheckServiceAffinity without services: the per (pod class, label set) table against the
    oracle's checkServiceAffinity on every node."""
    import ksim_ref as R
    from ksim import ingest
    from workloads import rnd_workload
    nodes, running, pods = rnd_workload(5, n_nodes=20, n_pods=60)
    for p in pods[::3]:
        p["spec"]["nodeSelector"] = {"tier": "a", "disk": "ssd"}
    cl = ingest.Cluster.from_objects(nodes, running, pods)
    ok, need = scheduler.service_affinity_table(cl.classes.items, cl.label_sets.items, ["disk", "region"])
    pred = R.new_service_affinity_predicate(["disk", "region"])
    infos = [R.NodeInfo(x) for x in sorted(nodes, key=lambda x: x["metadata"]["name"].encode())]
    assert need.any()
    for k, p in enumerate(pods):
        c = int(cl.pods["cls"][k])
        for i, ni in enumerate(infos):
            s = int(cl.cols["label_set"][i])
            assert bool((int(ok[c, s >> 5]) >> (s & 31)) & 1) == pred(p, ni)[0]
    pol = policy.decode({"predicates": [{"name": "CheckServiceAffinity", "argument": {"serviceAffinity": {"labels": ["disk"]}}},
                                        {"name": "PodFitsResources"}]})
    preds, _, _ = policy.key_sets(pol)
    assert "CheckServiceAffinity" in preds and policy.service_affinity_labels(pol) == ["disk"]
    assert scheduler.make_config(preds, []).predicates & abi.P_SERVICE_AFFINITY


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GPU_POLICIES))
def test_gpu_policy_arguments_through_cpp_front_end(name):
    """The Policy's arguments through the C++ front end (ksim_k8s_open_policy): CheckNodeLabelPresence,
    CheckServiceAffinity (no services), labelPreference / serviceAntiAffinity priorities evaluated in
    the library from raw fields — placements, FitError histograms' texts and lastNodeIndex equal the
    object oracle's."""
    import ctypes as C

    import numpy as np

    import ksim_ref as R
    from ksim import frontend
    from workloads import rnd_workload
    pol = policy.decode(GPU_POLICIES[name])
    preds, prios, lp = policy.key_sets(pol)
    sa = policy.service_affinity_labels(pol)
    args = policy.priority_arguments(pol)
    custom = {"CheckNodeLabelPresence": R.new_node_label_predicate(*lp)} if lp else {}
    if sa is not None:
        custom["CheckServiceAffinity"] = R.new_service_affinity_predicate(sa)
    cprios = {n: (R.node_label_priority(a[1], a[2]) if a[0] == "labelPreference" else R.service_anti_affinity_priority(a[1]))
              for n, a in args.items()}
    weights = dict(prios)
    label_prios = [(a[1], a[2] if a[0] == "labelPreference" else True, int(weights[n]), a[0] == "serviceAntiAffinity")
                   for n, a in args.items()]
    for seed in (3, 11):
        nodes, running, pods = rnd_workload(seed, n_nodes=31 + seed, n_pods=140)
        want, lni = R.simulate(nodes, running, pods, set(preds), list(prios), custom, custom_priorities=cprios)
        order = list(reversed(pods))
        cl = ingest.Cluster.from_objects(nodes, running, order)
        p = scheduler.plan(cl, preds, prios, label_presence=lp, custom_priorities=args, service_affinity=sa)
        fe = frontend.K8sCluster(nodes, running, order)
        h = fe.open_policy(p.cfg, prefer_avoid_weight=weights.get("NodePreferAvoidPodsPriority", 0),
                           image_locality_weight=weights.get("ImageLocalityPriority", 0), label_presence=lp,
                           service_affinity=sa, label_priorities=label_prios)
        n = len(order)
        out = np.zeros(n, np.int32)
        reasons = np.zeros((n, abi.NREASONS), np.int32)
        st = abi.Stats()
        try:
            h.call("ksim_schedule", 0, n, abi.vptr(out), abi.vptr(reasons), C.byref(st))
            ctr = C.c_uint64()
            h.call("ksim_get_counter", C.byref(ctr))
        finally:
            h.close()
        names = fe.names
        got = [(cl.pod_names[k], names[w] if w >= 0 else None,
                None if w >= 0 else scheduler.fit_error_message(len(names), reasons[k], cl.scalar_names.items))
               for k, w in enumerate(out)]
        assert got == want
        assert ctr.value == lni
