"""Inter-pod affinity → the device tables of ksim_load_affinity (include/ksim.h).

Reference semantics (paths under vendor/k8s.io/kubernetes/pkg/scheduler/):
- MatchInterPodAffinity: algorithm/predicates/predicates.go:1143-1450 with its metadata
  (getMatchingAntiAffinityTerms, :1235-1293; GetMetadata, predicates/metadata.go:102-123);
- InterPodAffinityPriority: algorithm/priorities/interpod_affinity.go:118-240;
- GetNamespacesFromPodAffinityTerm / PodMatchesTermsNamespaceAndSelector /
  NodesHaveSameTopologyKey: algorithm/priorities/util/topologies.go:28-71.

Every string test is resolved here, once per distinct object:
- a *selector* s is (namespaces, label selector) of one term as its defining pod resolves it;
  an *identity* is (namespace, labels) of a pod; ident_sel[i] has bit s when identity i matches s;
- a *topology key* k maps every node to a domain id (the node's value of label k interned, -1
  without it); two pseudo keys: ALL (every node in domain 0, for "a matching pod exists
  anywhere") and NODE (node i in domain i, for kubernetes.io/hostname terms, which only look at
  the node's own pods, predicates.go:1176-1179);
- a *counted pair* (s, k) keeps, per domain of k, the number of placed pods matching s: the
  pod-side terms read it (required affinity / anti-affinity, preferred terms);
- a *carried term* e is a term of a placed pod acting on later pods (existing pods'
  anti-affinity, the symmetric priority terms): per domain of its key, the summed weight (or,
  for required anti-affinity, the number) of placed pods carrying it.
Placing a pod adds one to every pair whose selector its identity matches and its carried
amounts to its node's domains (ksim_commit); removing subtracts.

Inputs whose reference behaviour is an error rather than a placement are rejected (Unsupported):
unparsable label selectors, required terms with an empty topologyKey, and running pods bound to
a node that is not in the snapshot while affinity terms exist (the reference then errors or
falls back to a metadata-less path).
"""
from __future__ import annotations

import json

import numpy as np

from . import abi, labels

HOSTNAME = "kubernetes.io/hostname"   # kubeletapis.LabelHostname
KEY_ALL, KEY_NODE = 0, 1              # pseudo keys
MAX_SEL = 65536
MAX_CARRY = 65536

TERM_DTYPE = np.dtype([("kind", "<i4"), ("pair", "<i4"), ("gate_key", "<i4"), ("exist_pair", "<i4"),
                       ("self_ok", "<i4"), ("pad", "<i4"), ("weight", "<i8")])
CARRY_DTYPE = np.dtype([("term", "<i4"), ("pad", "<i4"), ("amount", "<i8")])


class Unsupported(abi.KsimUnsupported):
    def __init__(self, msg):
        super().__init__(abi.E_UNSUPPORTED, msg)


def _canon(x):
    return json.dumps(x, sort_keys=True, separators=(",", ":"))


def _meta(o):
    return o.get("metadata") or {}


def _aff(p):
    return (p.get("spec") or {}).get("affinity") or {}


def has_pod_affinity(p):
    a = _aff(p)
    return a.get("podAffinity") is not None or a.get("podAntiAffinity") is not None


def _required(section):
    return list((section or {}).get("requiredDuringSchedulingIgnoredDuringExecution") or [])


def _preferred(section):
    return list((section or {}).get("preferredDuringSchedulingIgnoredDuringExecution") or [])


class _Interner:
    def __init__(self):
        self.ids, self.items = {}, []

    def get(self, key, item=None):
        i = self.ids.get(key)
        if i is None:
            i = self.ids[key] = len(self.items)
            self.items.append(key if item is None else item)
        return i


class _AnyOf:
    """A SelectorSpread selector: the pod's service / controller selectors, any of which counts a
    placed pod of its namespace that is not being deleted (selector_spreading.go:85-107)."""

    def __init__(self, sels):
        self.sels = tuple(sels)


ZONE_KEY = "\x00zone"   # pseudo key: utilnode.GetZoneKey (K/pkg/util/node/node.go), SelectorSpread's zones
PRESENCE = "\x00has:"   # pseudo key prefix: domain 0 on the nodes carrying the label


def zone_key_of(lab):
    """GetZoneKey: "" without both failure-domain labels, else region + ":\\x00:" + zone."""
    lab = lab or {}
    region = lab.get("failure-domain.beta.kubernetes.io/region", "")
    zone = lab.get("failure-domain.beta.kubernetes.io/zone", "")
    if region == "" and zone == "":
        return ""
    return region + ":\x00:" + zone


class AffinityIndex:
    """Collects the terms of every pod (running and queued), then builds the tables."""

    def __init__(self, node_labels, hard_weight=10):
        self.node_labels = node_labels            # per node (name-rank order): dict or None
        self.hard_weight = int(hard_weight)
        self.keys = _Interner()
        self.keys.get("\x00all")
        self.keys.get("\x00node")
        self.sels = _Interner()                   # (namespaces, selector) → (set, requirements)
        self.pairs = _Interner()                  # (sel, key)
        self.carry = _Interner()                  # (sel, key, kind)
        self.idents = _Interner()                 # (namespace, labels)
        self.aclasses = _Interner()               # → (required terms, preferred terms, carries, spread, aux)
        self.aux_key, self.aux_kind = None, abi.AUX_SPREAD   # the auxiliary priority (aux_pair), if any
        self.svc_labels = None                    # CheckServiceAffinity's labels (set_svc), if any
        self.svcs = _Interner()                   # service-affinity identities → (sel, pair_all, present, value)

    # ---------------------------------------------------------------- interning
    def _sel(self, defining_pod, term):
        nss = term.get("namespaces") or []
        ns = frozenset(nss) if nss else frozenset([_meta(defining_pod).get("namespace", "")])
        ps = term.get("labelSelector")
        try:
            sel = labels.from_label_selector(ps)
        except labels.SelectorError as e:
            raise Unsupported("pod %r: affinity label selector: %s" % (_meta(defining_pod).get("name"), e))
        key = (tuple(sorted(ns)), None if sel is labels.NOTHING else tuple(sel))
        return self.sels.get(key, (ns, sel)), sel

    def ident(self, pod):
        md = _meta(pod)
        deleting = md.get("deletionTimestamp") is not None
        return self.idents.get((md.get("namespace", ""), _canon(md.get("labels") or {}), deleting),
                               (md.get("namespace", ""), dict(md.get("labels") or {}), deleting))

    def _matches(self, ident_item, sel_item):
        ns, lab, deleting = ident_item
        nss, sel = sel_item
        if isinstance(sel, _AnyOf):
            return ns in nss and not deleting and any(labels.matches(x, lab) for x in sel.sels)
        return ns in nss and labels.matches(sel, lab)

    def spread_pair(self, pod, sels):
        """The counted pair (spread selector, node key) of a pod with SelectorSpread selectors."""
        if not sels:
            return -1
        ns = _meta(pod).get("namespace", "")
        key = ("\x00spread", ns, repr(list(sels)))
        s = self.sels.get(key, (frozenset([ns]), _AnyOf(sels)))
        self.keys.get(ZONE_KEY)
        return self.pairs.get((s, KEY_NODE))

    def set_aux(self, kind, key):
        """Configure the auxiliary counted priority (include/ksim.h ksim_affinity_tables.aux_*):
        kind abi.AUX_SPREAD (zones: key ZONE_KEY) or abi.AUX_SERVICE_ANTI (key: the label)."""
        self.aux_kind, self.aux_key = kind, key
        self.keys.get(key)

    def set_svc(self, affinity_labels):
        """CheckServiceAffinity's labels (include/ksim.h ksim_affinity_tables.svc_*): a value key and
        a presence key per label."""
        self.svc_labels = list(affinity_labels)
        for l in self.svc_labels:
            self.keys.get(l)
            self.keys.get(PRESENCE + l)

    def svc_class(self, pod, miss):
        """(identity, missing-label mask) of a pod a service selects whose nodeSelector lacks the
        labels of `miss`: the identity's selector is the pod's labels as a set selector in its
        namespace (serviceAffinityMetadataProducer, predicates.go:920-940: CreateSelectorFromLabels,
        FilterPodsByNamespace — deleting pods count), with the counted pairs the lender check reads."""
        md = _meta(pod)
        ns, lab = md.get("namespace", ""), md.get("labels") or {}
        key = (ns, _canon(lab))
        v = self.svcs.ids.get(key)
        if v is None:
            sel = labels.from_set(lab)
            s = self.sels.get(((ns,), tuple(sel)), (frozenset([ns]), sel))
            rec = (s, self.pairs.get((s, KEY_ALL)),
                   tuple(self.pairs.get((s, self.keys.ids[PRESENCE + l])) for l in self.svc_labels),
                   tuple(self.pairs.get((s, self.keys.ids[l])) for l in self.svc_labels))
            v = self.svcs.get(key, rec)
        return (v, int(miss))

    def aux_pair(self, pod, sels):
        """The pod's counted pair for the auxiliary priority, or -1: abi.AUX_SPREAD takes the
        services-only SelectorSpread selectors (any of them, not being deleted); abi.AUX_SERVICE_ANTI
        the one selecting service's selector as a plain set selector over the pod's namespace
        (filteredPod, selector_spreading.go:232-245: deleting pods count)."""
        if self.aux_key is None or not sels:
            return -1
        ns = _meta(pod).get("namespace", "")
        if self.aux_kind == abi.AUX_SPREAD:
            key = ("\x00spread", ns, repr(list(sels)))
            s = self.sels.get(key, (frozenset([ns]), _AnyOf(sels)))
        else:
            (sel,) = sels          # a ksim.labels selector (SpreadListers.selectors)
            s = self.sels.get(((ns,), tuple(sel)), (frozenset([ns]), sel))
        return self.pairs.get((s, KEY_NODE))

    def aclass(self, pod, spread_sels=(), aux_sels=(), svc=None):
        """The pod's own terms, carried terms, SelectorSpread pair, auxiliary pair and
        service-affinity identity (svc_class), interned; -1 when it has none of them."""
        sp = self.spread_pair(pod, spread_sels)
        ap = self.aux_pair(pod, aux_sels)
        if not has_pod_affinity(pod):
            return -1 if sp < 0 and ap < 0 and svc is None else self.aclasses.get(((), (), (), sp, ap, svc))
        a = _aff(pod)
        name = _meta(pod).get("name")
        req, pref, carries = [], [], {}
        my_ident = self.idents.items[self.ident(pod)]
        for kind, section in ((abi.AFF_REQ_AFFINITY, a.get("podAffinity")), (abi.AFF_REQ_ANTI, a.get("podAntiAffinity"))):
            for t in _required(section):
                key = t.get("topologyKey") or ""
                if not key:
                    raise Unsupported("pod %r: required pod (anti-)affinity term without topologyKey" % name)
                s, sel = self._sel(pod, t)
                if key == HOSTNAME:
                    mp = self.pairs.get((s, KEY_NODE))
                    gate, ep = self.keys.get(key), mp
                else:
                    k = self.keys.get(key)
                    mp, gate, ep = self.pairs.get((s, k)), k, self.pairs.get((s, KEY_ALL))
                self_ok = int(self._matches(my_ident, self.sels.items[s]))
                req.append((kind, mp, gate, ep, self_ok, 0))
        for sign, section in ((1, a.get("podAffinity")), (-1, a.get("podAntiAffinity"))):
            if section is None:
                continue
            for wt in _preferred(section):
                t = wt.get("podAffinityTerm") or {}
                s, sel = self._sel(pod, t)
                key = t.get("topologyKey") or ""
                if not key or sel is labels.NOTHING:
                    continue                              # matches no node / no pod: adds nothing
                pref.append((abi.AFF_PREFERRED, self.pairs.get((s, self.keys.get(key))), 0, 0, 0,
                             sign * int(wt.get("weight", 0))))

        def carry(t, kind, amount):
            s, sel = self._sel(pod, t)
            key = t.get("topologyKey") or ""
            if not key:
                if kind == abi.AFF_CARRY_ANTI:
                    raise Unsupported("pod %r: required anti-affinity term without topologyKey" % name)
                return                                    # NodesHaveSameTopologyKey is false
            if sel is labels.NOTHING:
                return
            e = self.carry.get((s, self.keys.get(key), kind))
            carries[e] = carries.get(e, 0) + amount

        for t in _required(a.get("podAntiAffinity")):
            carry(t, abi.AFF_CARRY_ANTI, 1)
        if a.get("podAffinity") is not None:
            if self.hard_weight > 0:
                for t in _required(a.get("podAffinity")):
                    carry(t, abi.AFF_CARRY_PRIO, self.hard_weight)
            for wt in _preferred(a.get("podAffinity")):
                carry(wt.get("podAffinityTerm") or {}, abi.AFF_CARRY_PRIO, int(wt.get("weight", 0)))
        if a.get("podAntiAffinity") is not None:
            for wt in _preferred(a.get("podAntiAffinity")):
                carry(wt.get("podAffinityTerm") or {}, abi.AFF_CARRY_PRIO, -int(wt.get("weight", 0)))
        carries = tuple(sorted((e, v) for e, v in carries.items() if v != 0 or self.carry.items[e][2] == abi.AFF_CARRY_ANTI))
        req.sort(key=lambda r: r[0] != abi.AFF_REQ_AFFINITY)   # affinity terms are checked before anti-affinity
        if not req and not pref and not carries and sp < 0 and ap < 0 and svc is None:
            return -1
        return self.aclasses.get((tuple(req), tuple(pref), carries, sp, ap, svc))

    # ------------------------------------------------------------------ tables
    def build(self, running_nodes, idents, aclasses):
        """(tables, remap): remap[interned identity] = ksim_pod.aff_ident (1 + table id, 0 when
        the identity matches no selector).  running_nodes: node ranks of the placed pods, whose
        interned identities / classes (-1: none) lead `idents` / `aclasses`."""
        if len(self.sels.items) > MAX_SEL:
            raise Unsupported("more than %d distinct inter-pod affinity selectors" % MAX_SEL)
        if len(self.carry.items) > MAX_CARRY:
            raise Unsupported("more than %d distinct carried inter-pod affinity terms" % MAX_CARRY)
        n = len(self.node_labels)
        K = len(self.keys.items)
        dom = np.full((K, n), -1, np.int32)
        n_dom = np.zeros(K, np.int32)
        dom[KEY_ALL, :] = 0
        n_dom[KEY_ALL] = 1
        dom[KEY_NODE, :] = np.arange(n, dtype=np.int32)
        n_dom[KEY_NODE] = n
        for k in range(2, K):
            name = self.keys.items[k]
            vals = {}
            for i, lab in enumerate(self.node_labels):
                if name == ZONE_KEY:
                    z = zone_key_of(lab)
                    if z != "":
                        dom[k, i] = vals.setdefault(z, len(vals))
                elif name.startswith(PRESENCE):
                    if lab is not None and name[len(PRESENCE):] in lab:
                        dom[k, i] = vals.setdefault(True, 0)
                elif lab is not None and name in lab:
                    dom[k, i] = vals.setdefault(lab[name], len(vals))
            n_dom[k] = len(vals)
        # identity masks (identities matching nothing become -1)
        I = len(self.idents.items)
        SW, CW = (len(self.sels.items) + 63) // 64, (len(self.carry.items) + 63) // 64
        isel = np.zeros((I, SW), np.uint64)
        ianti = np.zeros((I, CW), np.uint64)
        iprio = np.zeros((I, CW), np.uint64)
        for i, it in enumerate(self.idents.items):
            hit = [self._matches(it, si) for si in self.sels.items]
            for s, h in enumerate(hit):
                if h:
                    isel[i, s >> 6] |= np.uint64(1 << (s & 63))
            for e, (s, _, kind) in enumerate(self.carry.items):
                if hit[s]:
                    tgt = ianti if kind == abi.AFF_CARRY_ANTI else iprio
                    tgt[i, e >> 6] |= np.uint64(1 << (e & 63))
        live = (isel.any(axis=1) | ianti.any(axis=1) | iprio.any(axis=1)) if I else np.zeros(0, bool)
        remap = np.zeros(I, np.int32)     # ksim_pod.aff_ident: 1 + the table id, 0 = none
        remap[live] = np.arange(1, int(live.sum()) + 1, dtype=np.int32)
        # counted pairs / carried terms: offsets into the count arrays
        P = len(self.pairs.items)
        pair_sel = np.array([s for s, _ in self.pairs.items], np.int32)
        pair_key = np.array([k for _, k in self.pairs.items], np.int32)
        pair_off = np.zeros(P, np.int64)
        off = 0
        for c in range(P):
            pair_off[c] = off
            off += int(n_dom[pair_key[c]])
        cnt = np.zeros(max(off, 1), np.int32)
        E = len(self.carry.items)
        carry_key = np.array([k for _, k, _ in self.carry.items], np.int32)
        carry_kind = np.array([kd for _, _, kd in self.carry.items], np.int32)
        carry_sel = np.array([s for s, _, _ in self.carry.items], np.int32)
        carry_off = np.zeros(E, np.int64)
        off = 0
        for e in range(E):
            carry_off[e] = off
            off += int(n_dom[carry_key[e]])
        carried = np.zeros(max(off, 1), np.int64)
        # affinity classes
        A = len(self.aclasses.items)
        terms, carries = [], []
        ac = np.zeros((A, 6), np.int32)   # req_off, req_cnt, pref_off, pref_cnt, carry_off, carry_cnt
        spread_pair = np.array([x[3] for x in self.aclasses.items], np.int32) if A else np.zeros(0, np.int32)
        aux_pair = np.array([x[4] for x in self.aclasses.items], np.int32) if A else np.zeros(0, np.int32)
        for a, (req, pref, car, _, _, _) in enumerate(self.aclasses.items):
            ac[a, 0], ac[a, 1] = len(terms), len(req)
            terms.extend(req)
            ac[a, 2], ac[a, 3] = len(terms), len(pref)
            terms.extend(pref)
            ac[a, 4], ac[a, 5] = len(carries), len(car)
            carries.extend(car)
        terms_a = np.zeros(max(len(terms), 1), TERM_DTYPE)
        for j, t in enumerate(terms):
            terms_a[j] = t[:5] + (0, t[5])
        carries_a = np.zeros(max(len(carries), 1), CARRY_DTYPE)
        for j, (e, v) in enumerate(carries):
            carries_a[j] = (e, 0, v)
        # the running pods' contribution (NodeInfo.AddPod of every cached pod)
        for w, i_id, a_id in zip(running_nodes, idents[:len(running_nodes)], aclasses[:len(running_nodes)]):
            for c in range(P):
                s = int(pair_sel[c])
                if (int(isel[i_id, s >> 6]) >> (s & 63)) & 1:
                    d = dom[pair_key[c], w]
                    if d >= 0:
                        cnt[pair_off[c] + d] += 1
            if a_id >= 0:
                for j in range(ac[a_id, 4], ac[a_id, 4] + ac[a_id, 5]):
                    e, v = int(carries_a[j]["term"]), int(carries_a[j]["amount"])
                    d = dom[carry_key[e], w]
                    if d >= 0:
                        carried[carry_off[e] + d] += v
        return dict(n_keys=K, n_sel=len(self.sels.items), n_ident=int(live.sum()), n_pair=P, n_carry=E, n_aclass=A,
                    sel_words=SW, carry_words=CW,
                    n_nodes=n, hard_weight=self.hard_weight, dom=np.ascontiguousarray(dom), n_dom=n_dom,
                    ident_sel=isel[live].copy(), ident_anti=ianti[live].copy(), ident_prio=iprio[live].copy(),
                    pair_sel=pair_sel, pair_key=pair_key, pair_off=pair_off, carry_key=carry_key,
                    carry_kind=carry_kind, carry_sel=carry_sel, carry_off=carry_off,
                    ac=np.ascontiguousarray(ac), terms=terms_a, carries=carries_a, cnt=cnt, carried=carried,
                    zone_key=self.keys.ids.get(ZONE_KEY, -1), spread_pair=spread_pair,
                    aux_pair=aux_pair if self.aux_key is not None else None,
                    aux_key=self.keys.ids[self.aux_key] if self.aux_key is not None else -1, aux_kind=self.aux_kind,
                    aux_weight=0, n_terms=len(terms), n_carries=len(carries),
                    **self._svc_tables(isel, live, remap, dom, running_nodes, idents)), remap


def _svc_tables_impl(self, isel, live, remap, dom, running_nodes, idents):
    """CheckServiceAffinity's lender tables (include/ksim.h ksim_affinity_tables.svc_*): per identity
    its pairs, per affinity class its identity and missing labels, per live affinity identity the
    service-affinity identities whose selector it matches, and the running pods' disagreements."""
    if self.svc_labels is None:
        return dict(svc_on=False)
    V, L = len(self.svcs.items), len(self.svc_labels)
    rec = np.zeros(V, abi.SVC_IDENT_DTYPE)
    for v, (_, pall, pres, pval) in enumerate(self.svcs.items):
        rec[v]["pair_all"] = pall
        rec[v]["pair_present"][:L] = pres
        rec[v]["pair_value"][:L] = pval
    A = len(self.aclasses.items)
    svc_class = np.full(max(A, 1), -1, np.int32)
    svc_miss = np.zeros(max(A, 1), np.uint32)
    for a, it in enumerate(self.aclasses.items):
        if it[5] is not None:
            svc_class[a], svc_miss[a] = it[5]
    sel_of = [s for s, _, _, _ in self.svcs.items]
    live_ids = np.nonzero(live)[0] if len(live) else np.zeros(0, np.int64)
    off, lst = [0], []
    for i in live_ids:
        for v, s in enumerate(sel_of):
            if (int(isel[i, s >> 6]) >> (s & 63)) & 1:
                lst.append(v)
        off.append(len(lst))
    # the running pods' nodes: per identity, the (present, value) of every label must agree
    conflict = np.zeros(max(V, 1), np.uint32)
    vkeys = [self.keys.ids[l] for l in self.svc_labels]
    for v, s in enumerate(sel_of):
        seen = [set() for _ in range(L)]
        for w, i_id in zip(running_nodes, idents[:len(running_nodes)]):
            if (int(isel[i_id, s >> 6]) >> (s & 63)) & 1:
                for l in range(L):
                    seen[l].add(int(dom[vkeys[l], w]))
        for l in range(L):
            if len(seen[l]) > 1:
                conflict[v] |= np.uint32(1 << l)
    return dict(svc_on=True, n_svc=V, n_svc_labels=L, svc_ident=rec, svc_class=svc_class, svc_miss=svc_miss,
                svc_conflict=conflict, svc_of_off=np.array(off, np.int32), svc_of=np.array(lst or [0], np.int32))


AffinityIndex._svc_tables = _svc_tables_impl


def tables_struct(d):
    """ksim_affinity_tables over a tables dict (the dict keeps the arrays alive)."""
    t = abi.AffinityTables()
    for k in ("n_keys", "n_sel", "n_ident", "n_pair", "n_carry", "n_aclass", "hard_weight", "sel_words", "carry_words",
              "zone_key"):
        setattr(t, k, int(d[k]))
    t.n_nodes = int(d["n_nodes"])
    for name, ct in (("dom", abi.C.c_int32), ("n_dom", abi.C.c_int32), ("ident_sel", abi.C.c_uint64),
                     ("ident_anti", abi.C.c_uint64), ("ident_prio", abi.C.c_uint64), ("pair_sel", abi.C.c_int32),
                     ("pair_key", abi.C.c_int32), ("pair_off", abi.C.c_int64), ("carry_key", abi.C.c_int32),
                     ("carry_kind", abi.C.c_int32), ("carry_off", abi.C.c_int64), ("ac", abi.C.c_int32),
                     ("cnt", abi.C.c_int32), ("carried", abi.C.c_int64), ("spread_pair", abi.C.c_int32)):
        d[name] = np.ascontiguousarray(d[name])
        setattr(t, name, abi.ptr(d[name], ct))
    d["terms"] = np.ascontiguousarray(d["terms"])
    d["carries"] = np.ascontiguousarray(d["carries"])
    t.terms = d["terms"].ctypes.data_as(abi.C.c_void_p)
    t.carries = d["carries"].ctypes.data_as(abi.C.c_void_p)
    if d.get("svc_on") and d.get("svc_use", True):
        for k, dt in (("svc_class", np.int32), ("svc_miss", np.uint32), ("svc_conflict", np.uint32),
                      ("svc_of_off", np.int32), ("svc_of", np.int32)):
            d[k] = np.ascontiguousarray(d[k], dt)
        d["svc_ident"] = np.ascontiguousarray(d["svc_ident"])
        t.n_svc, t.n_svc_labels = int(d["n_svc"]), int(d["n_svc_labels"])
        t.svc_ident = d["svc_ident"].ctypes.data_as(abi.C.c_void_p)
        t.svc_class = abi.ptr(d["svc_class"], abi.C.c_int32)
        t.svc_miss = abi.ptr(d["svc_miss"], abi.C.c_uint32)
        t.svc_conflict = abi.ptr(d["svc_conflict"], abi.C.c_uint32)
        t.svc_of_off = abi.ptr(d["svc_of_off"], abi.C.c_int32)
        t.svc_of = abi.ptr(d["svc_of"], abi.C.c_int32)
    if d.get("aux_pair") is not None and int(d.get("aux_weight", 0)):
        d["aux_pair"] = np.ascontiguousarray(d["aux_pair"], np.int32)
        t.aux_pair = abi.ptr(d["aux_pair"], abi.C.c_int32)
        t.aux_key, t.aux_kind, t.aux_weight = int(d["aux_key"]), int(d["aux_kind"]), int(d["aux_weight"])
    else:
        t.aux_key = -1
    t.n_terms = int(d.get("n_terms", len(d["terms"])))       # the arrays are padded to one entry
    t.n_carries = int(d.get("n_carries", len(d["carries"])))
    t.cnt_len = len(d["cnt"])
    t.carried_len = len(d["carried"])
    return t
