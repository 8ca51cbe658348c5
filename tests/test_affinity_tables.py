"""The inter-pod affinity tables (ksim/affinity.py → ksim_load_affinity) read the way the kernels
read them (ksim_common.h: ksim_interpod_pred, ksim_interpod_raw, ksim_interpod_score,
ksim_aff_commit), checked on the CPU against the oracle's object-level restatement
(ksim_ref.interpod_affinity_matches / interpod_affinity_priority) pod by pod through whole
simulations: before each pod every node's predicate reasons and normalised priority score must
agree; the pod is then placed where the oracle's scheduler puts it and committed to the tables."""
import numpy as np
import pytest

import ksim_ref as R
from ksim import abi, ingest, scheduler
from workloads import rnd_affinity_workload

REASON_BITS = {R.R_AFFINITY: abi.R_POD_AFFINITY, R.R_EXISTING_ANTI: abi.R_EXISTING_ANTI,
               R.R_AFFINITY_RULES: abi.R_AFFINITY_RULES, R.R_ANTI_AFFINITY_RULES: abi.R_ANTI_AFFINITY_RULES}


class TableModel:
    """The device's view of the tables (mutable counts)."""

    def __init__(self, T):
        self.T = T
        self.cnt = T["cnt"].astype(np.int64).copy()
        self.carried = T["carried"].copy()

    @staticmethod
    def bits(words):
        return [64 * w + b for w, x in enumerate(words) for b in range(64) if (int(x) >> b) & 1]

    def dom(self, k, i):
        return int(self.T["dom"][k, i])

    def pair_hit(self, c, i):
        d = self.dom(self.T["pair_key"][c], i)
        return d >= 0 and self.cnt[self.T["pair_off"][c] + d] > 0

    def pred(self, ident, acl, i):
        T = self.T
        if ident > 0:
            for e in self.bits(T["ident_anti"][ident - 1]):
                d = self.dom(T["carry_key"][e], i)
                if d >= 0 and self.carried[T["carry_off"][e] + d] > 0:
                    return (1 << abi.R_POD_AFFINITY) | (1 << abi.R_EXISTING_ANTI)
        if acl <= 0:
            return 0
        ac = T["ac"][acl - 1]
        for t in T["terms"][ac[0]:ac[0] + ac[1]]:
            match = self.dom(t["gate_key"], i) >= 0 and self.pair_hit(t["pair"], i)
            if t["kind"] == abi.AFF_REQ_AFFINITY:
                if not match and (not t["self_ok"] or self.pair_hit(t["exist_pair"], i)):
                    return (1 << abi.R_POD_AFFINITY) | (1 << abi.R_AFFINITY_RULES)
            elif match:
                return (1 << abi.R_POD_AFFINITY) | (1 << abi.R_ANTI_AFFINITY_RULES)
        return 0

    def raw(self, ident, acl, i):
        T, s = self.T, 0
        if acl > 0:
            ac = T["ac"][acl - 1]
            for t in T["terms"][ac[2]:ac[2] + ac[3]]:
                d = self.dom(T["pair_key"][t["pair"]], i)
                if d >= 0:
                    s += int(t["weight"]) * int(self.cnt[T["pair_off"][t["pair"]] + d])
        if ident > 0:
            for e in self.bits(T["ident_prio"][ident - 1]):
                d = self.dom(T["carry_key"][e], i)
                if d >= 0:
                    s += int(self.carried[T["carry_off"][e] + d])
        return s

    def commit(self, ident, acl, w, sign=1):
        T = self.T
        if ident > 0:
            sm = set(self.bits(T["ident_sel"][ident - 1]))
            for c in range(T["n_pair"]):
                if int(T["pair_sel"][c]) in sm:
                    d = self.dom(T["pair_key"][c], w)
                    if d >= 0:
                        self.cnt[T["pair_off"][c] + d] += sign
        if acl > 0:
            ac = T["ac"][acl - 1]
            for k in T["carries"][ac[4]:ac[4] + ac[5]]:
                d = self.dom(T["carry_key"][k["term"]], w)
                if d >= 0:
                    self.carried[T["carry_off"][k["term"]] + d] += sign * int(k["amount"])


def _score(raw, mn, mx):
    return int(10.0 * ((raw - mn) / (mx - mn))) if mx - mn > 0 else 0


@pytest.mark.parametrize("seed", range(6))
def test_tables_match_oracle_through_a_simulation(seed):
    nodes, running, pods = rnd_affinity_workload(seed, n_nodes=14 + seed, n_pods=50, n_running=10)
    order = list(reversed(pods))
    cl = ingest.Cluster.from_objects(nodes, running, order)
    assert cl.affinity is not None
    model = TableModel(cl.affinity)
    by_name = {n: i for i, n in enumerate(cl.names)}
    infos = [R.NodeInfo(x) for x in sorted(nodes, key=lambda x: x["metadata"]["name"].encode())]
    for p in running:
        infos[by_name[p["spec"]["nodeName"]]].add_pod(p)
    keys, prios = R.provider("DefaultProvider")
    sched = R.GenericScheduler(keys, prios)
    for k, pod in enumerate(order):
        ident, acl = int(cl.pods[k]["aff_ident"]), int(cl.pods[k]["aff_class"])
        aff_pods = [(p, ni.node) for ni in infos for p in ni.pods_with_affinity]
        meta = R.matching_anti_affinity_terms(pod, aff_pods)
        all_pods = [(p, ni.node) for ni in infos for p in ni.pods]
        fit = []
        for i, ni in enumerate(infos):
            ok, reasons, err = R.interpod_affinity_matches(pod, ni.node, meta, all_pods, [(q, ni.node) for q in ni.pods])
            assert err is None
            want = 0
            for r in reasons:
                want |= 1 << REASON_BITS[r]
            assert model.pred(ident, acl, i) == want, (pod["metadata"]["name"], cl.names[i])
            if ok:
                fit.append(i)
        if len(fit) > 1:
            want = R.interpod_affinity_priority(pod, infos, [infos[i].node for i in fit], 10)
            raws = [model.raw(ident, acl, i) for i in fit]
            mn, mx = min([0] + raws), max([0] + raws)
            assert [_score(r, mn, mx) for r in raws] == want, pod["metadata"]["name"]
        try:
            host = sched.schedule(pod, infos)
        except R.FitError:
            continue
        w = by_name[host]
        infos[w].add_pod(dict(pod, spec=dict(pod["spec"], nodeName=host)))
        model.commit(ident, acl, w)


def test_remove_undoes_commit():
    nodes, running, pods = rnd_affinity_workload(11, n_nodes=10, n_pods=20)
    cl = ingest.Cluster.from_objects(nodes, running, pods)
    m = TableModel(cl.affinity)
    before = (m.cnt.copy(), m.carried.copy())
    for k in range(len(pods)):
        m.commit(int(cl.pods[k]["aff_ident"]), int(cl.pods[k]["aff_class"]), k % 10)
    for k in range(len(pods)):
        m.commit(int(cl.pods[k]["aff_ident"]), int(cl.pods[k]["aff_class"]), k % 10, -1)
    assert np.array_equal(m.cnt, before[0]) and np.array_equal(m.carried, before[1])


def test_pods_without_terms_take_no_part():
    nodes, running, pods = rnd_affinity_workload(3, n_nodes=6, n_pods=10, p_aff=0.0, n_running=0)
    assert ingest.Cluster.from_objects(nodes, running, pods).affinity is None
    p = scheduler.provider("DefaultProvider")
    assert scheduler.make_config(*p).predicates & abi.P_INTERPOD_AFFINITY
    assert scheduler.make_config(*p).weights[abi.W_INTERPOD] == 1
