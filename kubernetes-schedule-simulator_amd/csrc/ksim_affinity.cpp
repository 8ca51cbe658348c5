// ksim_affinity.cpp — ksim_load_affinity: validates and uploads the inter-pod affinity tables
// (layout in include/ksim.h; built by ksim/affinity.py) that MatchInterPodAffinity
// (predicates.go:1143-1450) and InterPodAffinityPriority (interpod_affinity.go:118-240) read on
// the device (ksim_common.h ksim_interpod_pred / ksim_interpod_raw / ksim_aff_commit).
//
// Every index the kernels follow is checked here against the array it indexes, so a malformed
// table is a KSIM_E_INVAL on the host, never an out-of-bounds access on the device.
#include "ksim_handle.h"

namespace {

bool bad_range(int64_t off, int64_t cnt, int64_t len) { return off < 0 || cnt < 0 || off + cnt > len; }

int validate(ksim_handle* h, const ksim_affinity_tables* t) {
  const int64_t n = h->ctx.n;
  if (t->n_nodes != n) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: tables for %lld nodes, table has %lld",
                                        (long long)t->n_nodes, (long long)n);
  if (t->n_keys < 2 || t->n_sel < 0 || t->n_ident < 0 || t->n_pair < 0 || t->n_carry < 0 || t->n_aclass < 0 ||
      t->n_terms < 0 || t->n_carries < 0 || t->cnt_len < 0 || t->carried_len < 0)
    return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: negative size (or fewer than the two pseudo keys)");
  if (t->n_sel > KSIM_AFF_MAX_SEL || t->n_carry > KSIM_AFF_MAX_CARRY)
    return ksim_fail(h, KSIM_E_UNSUPPORTED, "ksim_load_affinity: more than %d selectors or %d carried terms",
                     KSIM_AFF_MAX_SEL, KSIM_AFF_MAX_CARRY);
  if (t->sel_words != (t->n_sel + 63) / 64 || t->carry_words != (t->n_carry + 63) / 64)
    return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: sel_words / carry_words do not match n_sel / n_carry");
  const int64_t SW = t->sel_words, CW = t->carry_words;
  auto need = [&](const void* p, int64_t cnt) { return cnt == 0 || p != nullptr; };
  if (!need(t->dom, (int64_t)t->n_keys * n) || !t->n_dom || !need(t->ident_sel, t->n_ident * SW) ||
      !need(t->ident_anti, t->n_ident * CW) || !need(t->ident_prio, t->n_ident * CW) || !need(t->pair_sel, t->n_pair) ||
      !need(t->pair_key, t->n_pair) || !need(t->pair_off, t->n_pair) || !need(t->carry_key, t->n_carry) ||
      !need(t->carry_kind, t->n_carry) || !need(t->carry_off, t->n_carry) || !need(t->ac, 6 * (int64_t)t->n_aclass) ||
      !need(t->terms, t->n_terms) || !need(t->carries, t->n_carries) || !need(t->cnt, t->cnt_len) ||
      !need(t->carried, t->carried_len))
    return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: missing array");
  for (int32_t k = 0; k < t->n_keys; ++k) {
    const int32_t D = t->n_dom[k];
    if (D < 0) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: key %d has a negative domain count", k);
    const int32_t* row = t->dom + (int64_t)k * n;
    for (int64_t i = 0; i < n; ++i)
      if (row[i] < -1 || row[i] >= D) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: dom[%d][%lld] out of range", k, (long long)i);
  }
  // the bits an identity may set: selectors that exist, carried terms of the matching kind
  std::vector<uint64_t> sel_mask(SW, 0), anti_mask(CW, 0), prio_mask(CW, 0);
  for (int32_t s = 0; s < t->n_sel; ++s) sel_mask[s >> 6] |= 1ull << (s & 63);
  for (int32_t e = 0; e < t->n_carry; ++e) {
    const int32_t k = t->carry_key[e];
    if (k < 0 || k >= t->n_keys || bad_range(t->carry_off[e], t->n_dom[k], t->carried_len))
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: carried term %d out of range", e);
    if (t->carry_kind[e] == KSIM_AFF_CARRY_ANTI) anti_mask[e >> 6] |= 1ull << (e & 63);
    else if (t->carry_kind[e] == KSIM_AFF_CARRY_PRIO) prio_mask[e >> 6] |= 1ull << (e & 63);
    else return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: carried term %d has an unknown kind", e);
  }
  for (int64_t i = 0; i < t->n_ident; ++i) {
    for (int64_t w = 0; w < SW; ++w)
      if (t->ident_sel[i * SW + w] & ~sel_mask[w])
        return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: identity %lld names a selector out of range", (long long)i);
    for (int64_t w = 0; w < CW; ++w)
      if ((t->ident_anti[i * CW + w] & ~anti_mask[w]) || (t->ident_prio[i * CW + w] & ~prio_mask[w]))
        return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: identity %lld names a carried term out of range", (long long)i);
  }
  for (int32_t c = 0; c < t->n_pair; ++c) {
    const int32_t k = t->pair_key[c];
    if (t->pair_sel[c] < 0 || t->pair_sel[c] >= t->n_sel || k < 0 || k >= t->n_keys ||
        bad_range(t->pair_off[c], t->n_dom[k], t->cnt_len))
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: counted pair %d out of range", c);
  }
  for (int32_t j = 0; j < t->n_terms; ++j) {
    const ksim_aff_term& x = t->terms[j];
    if (x.kind < KSIM_AFF_REQ_AFFINITY || x.kind > KSIM_AFF_PREFERRED || x.pair < 0 || x.pair >= t->n_pair)
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: term %d out of range", j);
    if (x.kind != KSIM_AFF_PREFERRED &&
        (x.gate_key < 0 || x.gate_key >= t->n_keys || (x.kind == KSIM_AFF_REQ_AFFINITY && (x.exist_pair < 0 || x.exist_pair >= t->n_pair))))
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: required term %d out of range", j);
  }
  for (int32_t j = 0; j < t->n_carries; ++j)
    if (t->carries[j].term < 0 || t->carries[j].term >= t->n_carry)
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: carry entry %d out of range", j);
  for (int32_t a = 0; a < t->n_aclass; ++a) {
    const int32_t* r = t->ac + 6 * (int64_t)a;
    if (bad_range(r[0], r[1], t->n_terms) || bad_range(r[2], r[3], t->n_terms) || bad_range(r[4], r[5], t->n_carries))
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: class %d ranges out of bounds", a);
    for (int32_t j = r[0]; j < r[0] + r[1]; ++j)
      if (t->terms[j].kind == KSIM_AFF_PREFERRED)
        return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: class %d lists a preferred term among its required ones", a);
    for (int32_t j = r[2]; j < r[2] + r[3]; ++j)
      if (t->terms[j].kind != KSIM_AFF_PREFERRED)
        return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: class %d lists a required term among its preferred ones", a);
  }
  if (t->zone_key < -1 || t->zone_key >= t->n_keys)
    return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: zone key out of range");
  if (t->aux_pair) {
    if (t->aux_key < 0 || t->aux_key >= t->n_keys || (t->aux_kind != KSIM_AUX_SPREAD && t->aux_kind != KSIM_AUX_SERVICE_ANTI) ||
        t->aux_weight < 0)
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: auxiliary priority key / kind / weight out of range");
    for (int32_t a = 0; a < t->n_aclass; ++a) {
      const int32_t c = t->aux_pair[a];
      if (c < -1 || c >= t->n_pair || (c >= 0 && t->pair_key[c] != 1))
        return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: class %d auxiliary pair out of range", a);
    }
  }
  if (t->spread_pair)
    for (int32_t a = 0; a < t->n_aclass; ++a) {
      const int32_t c = t->spread_pair[a];
      // the scan reads the pair's count at the node's own index: it must be on the node pseudo key
      if (c < -1 || c >= t->n_pair || (c >= 0 && t->pair_key[c] != 1))
        return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: class %d spread pair out of range", a);
    }
  if (t->svc_class) {
    if (!t->svc_ident || !t->svc_miss || !t->svc_conflict || !t->svc_of_off || t->n_svc < 0 || t->n_svc_labels < 0 ||
        t->n_svc_labels > KSIM_SVC_LABELS)
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: service-affinity tables incomplete");
    for (int32_t a = 0; a < t->n_aclass; ++a)
      if (t->svc_class[a] < -1 || t->svc_class[a] >= t->n_svc || (t->svc_miss[a] >> t->n_svc_labels) != 0)
        return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: class %d service-affinity identity out of range", a);
    auto pair_on = [&](int32_t c, bool node_key) {  // a pair on a real key (the key-0 pair on key 0)
      return c >= 0 && c < t->n_pair && (node_key ? t->pair_key[c] == 0 : t->pair_key[c] >= 2);
    };
    for (int32_t v = 0; v < t->n_svc; ++v) {
      const ksim_svc_ident& S = t->svc_ident[v];
      bool ok = pair_on(S.pair_all, true);
      for (int32_t l = 0; l < t->n_svc_labels && ok; ++l) ok = pair_on(S.pair_present[l], false) && pair_on(S.pair_value[l], false);
      if (!ok) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: service-affinity identity %d pairs out of range", v);
    }
    if (t->svc_of_off[0] != 0)
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: svc_of_off[0] must be 0");
    for (int32_t i = 0; i < t->n_ident; ++i)
      if (t->svc_of_off[i + 1] < t->svc_of_off[i] || (t->svc_of_off[i + 1] > t->svc_of_off[i] && !t->svc_of))
        return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: svc_of_off not ascending");
    for (int32_t e = 0; e < t->svc_of_off[t->n_ident]; ++e)
      if (t->svc_of[e] < 0 || t->svc_of[e] >= t->n_svc)
        return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: svc_of entry %d out of range", e);
  }
  for (size_t q = 0; q < h->q_ident.size(); ++q)
    if (h->q_ident[q] > t->n_ident || h->q_aclass[q] > t->n_aclass)
      return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: queued pod %zu uses an identity / class beyond the tables", q);
  return KSIM_OK;
}

}  // namespace

extern "C" int ksim_load_affinity(ksim_handle* h, const ksim_affinity_tables* t) {
  if (!h || !t) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_affinity: null argument");
  if (!h->have_nodes) return ksim_fail(h, KSIM_E_STATE, "ksim_load_affinity: load the node table first");
  HIPCHK(h, hipSetDevice(h->device));
  int rc = validate(h, t);
  if (rc) return rc;
  const int64_t n = h->ctx.n;
  const size_t nb0 = h->bufs.size();
  KsimAff A{};
  int32_t *dom, *ps, *pk, *ck, *ac, *cnt;
  uint64_t *is, *ia, *ip;
  int64_t *po, *co, *carried, *mm, *part, *zsum, *zread;
  int32_t* spair = nullptr;
  int32_t* apair = nullptr;
  int64_t *asum = nullptr, *aread = nullptr;
  int32_t *sv_cls = nullptr, *sv_of_off = nullptr, *sv_of = nullptr;
  uint32_t *sv_miss = nullptr, *sv_conf = nullptr;
  ksim_svc_ident* sv = nullptr;
  ksim_aff_term* terms;
  ksim_aff_carry* carries;
  uint32_t* ticket;
  const int64_t grid_max = n / KSIM_BLOCK + 1;  // the widest launch (one node per lane)
  if ((rc = dev_upload(h, &dom, t->dom, (size_t)t->n_keys * n)) || (rc = dev_upload(h, &is, t->ident_sel, (size_t)t->n_ident * t->sel_words)) ||
      (rc = dev_upload(h, &ia, t->ident_anti, (size_t)t->n_ident * t->carry_words)) ||
      (rc = dev_upload(h, &ip, t->ident_prio, (size_t)t->n_ident * t->carry_words)) ||
      (rc = dev_upload(h, &ps, t->pair_sel, t->n_pair)) || (rc = dev_upload(h, &pk, t->pair_key, t->n_pair)) ||
      (rc = dev_upload(h, &po, t->pair_off, t->n_pair)) || (rc = dev_upload(h, &ck, t->carry_key, t->n_carry)) ||
      (rc = dev_upload(h, &co, t->carry_off, t->n_carry)) || (rc = dev_upload(h, &ac, t->ac, 6 * (size_t)t->n_aclass)) ||
      (rc = dev_upload(h, &terms, t->terms, t->n_terms)) || (rc = dev_upload(h, &carries, t->carries, t->n_carries)) ||
      (rc = dev_upload(h, &cnt, t->cnt, t->cnt_len)) || (rc = dev_upload(h, &carried, t->carried, t->carried_len)) ||
      (rc = dev_upload<int64_t>(h, &mm, nullptr, KSIM_AFF_MM)) ||
      (rc = dev_upload<int64_t>(h, &part, nullptr, KSIM_AFF_PART * (size_t)grid_max)) ||
      (rc = dev_upload<uint32_t>(h, &ticket, nullptr, 4)))
    return rc;
  const int32_t n_zone = t->zone_key >= 0 ? t->n_dom[t->zone_key] : 0;
  if ((rc = dev_upload<int64_t>(h, &zsum, nullptr, n_zone)) || (rc = dev_upload<int64_t>(h, &zread, nullptr, n_zone)))
    return rc;
  if (t->spread_pair && (rc = dev_upload(h, &spair, t->spread_pair, t->n_aclass))) return rc;
  const int32_t n_adom = t->aux_pair ? t->n_dom[t->aux_key] : 0;
  if (t->svc_class &&
      ((rc = dev_upload(h, &sv_cls, t->svc_class, t->n_aclass)) || (rc = dev_upload(h, &sv_miss, t->svc_miss, t->n_aclass)) ||
       (rc = dev_upload(h, &sv, t->svc_ident, t->n_svc)) || (rc = dev_upload(h, &sv_conf, t->svc_conflict, t->n_svc)) ||
       (rc = dev_upload(h, &sv_of_off, t->svc_of_off, (size_t)t->n_ident + 1)) ||
       (rc = dev_upload(h, &sv_of, t->svc_of, (size_t)t->svc_of_off[t->n_ident]))))
    return rc;
  if (t->aux_pair && ((rc = dev_upload(h, &apair, t->aux_pair, t->n_aclass)) ||
                      (rc = dev_upload<int64_t>(h, &asum, nullptr, n_adom)) || (rc = dev_upload<int64_t>(h, &aread, nullptr, n_adom))))
    return rc;
  // node-like keys: every domain holds at most one node (the node pseudo key, a unique hostname
  // label), so a commit changes one row's counts; other keys' domains are shared by several nodes
  std::vector<uint8_t> nodelike(t->n_keys, 1);
  for (int32_t k = 0; k < t->n_keys; ++k) {
    std::vector<int32_t> per(t->n_dom[k], 0);
    const int32_t* row = t->dom + (int64_t)k * n;
    for (int64_t i = 0; i < n && nodelike[k]; ++i)
      if (row[i] >= 0 && ++per[row[i]] > 1) nodelike[k] = 0;
  }
  std::vector<uint8_t> ishared(t->n_ident, 0), ashared(t->n_aclass, 0);
  for (int64_t i = 0; i < t->n_ident; ++i)
    for (int32_t cp = 0; cp < t->n_pair && !ishared[i]; ++cp) {
      const int32_t s = t->pair_sel[cp];
      if (((t->ident_sel[i * t->sel_words + (s >> 6)] >> (s & 63)) & 1ull) && !nodelike[t->pair_key[cp]]) ishared[i] = 1;
    }
  for (int32_t a = 0; a < t->n_aclass; ++a) {
    const int32_t* r = t->ac + 6 * (int64_t)a;
    for (int32_t j = r[4]; j < r[4] + r[5]; ++j)
      if (!nodelike[t->carry_key[t->carries[j].term]]) ashared[a] = 1;
  }
  uint8_t *ish, *ash;
  if ((rc = dev_upload(h, &ish, ishared.data(), ishared.size())) || (rc = dev_upload(h, &ash, ashared.data(), ashared.size())))
    return rc;
  // per identity, as lists (the general persistent kernel's pod-context records): the carried
  // anti-affinity / priority terms it matches and the counted pairs (with their key) it matches
  std::vector<int32_t> anti_off(1, 0), prio_off(1, 0), mp_off(1, 0), anti, prio, mp;
  int32_t mx_anti = 0, mx_prio = 0, mx_mp = 0;
  for (int64_t i = 0; i < t->n_ident; ++i) {
    for (int32_t w = 0; w < t->carry_words; ++w) {
      for (uint64_t m = t->ident_anti[i * t->carry_words + w]; m; m &= m - 1) anti.push_back(64 * w + __builtin_ctzll(m));
      for (uint64_t m = t->ident_prio[i * t->carry_words + w]; m; m &= m - 1) prio.push_back(64 * w + __builtin_ctzll(m));
    }
    for (int32_t cp = 0; cp < t->n_pair; ++cp) {
      const int32_t s = t->pair_sel[cp];
      if ((t->ident_sel[i * t->sel_words + (s >> 6)] >> (s & 63)) & 1ull) { mp.push_back(cp); mp.push_back(t->pair_key[cp]); }
    }
    mx_anti = std::max<int32_t>(mx_anti, (int32_t)anti.size() - anti_off.back());
    mx_prio = std::max<int32_t>(mx_prio, (int32_t)prio.size() - prio_off.back());
    mx_mp = std::max<int32_t>(mx_mp, ((int32_t)mp.size() - mp_off.back()) / 2);
    anti_off.push_back((int32_t)anti.size());
    prio_off.push_back((int32_t)prio.size());
    mp_off.push_back((int32_t)mp.size() / 2);
  }
  int32_t mx_req = 0, mx_pref = 0, mx_car = 0;
  for (int32_t a = 0; a < t->n_aclass; ++a) {
    mx_req = std::max(mx_req, t->ac[6 * (int64_t)a + 1]);
    mx_pref = std::max(mx_pref, t->ac[6 * (int64_t)a + 3]);
    mx_car = std::max(mx_car, t->ac[6 * (int64_t)a + 5]);
  }
  int32_t *dao, *da, *dpo, *dp, *dmo, *dm;
  if ((rc = dev_upload(h, &dao, anti_off.data(), anti_off.size())) || (rc = dev_upload(h, &da, anti.data(), anti.size())) ||
      (rc = dev_upload(h, &dpo, prio_off.data(), prio_off.size())) || (rc = dev_upload(h, &dp, prio.data(), prio.size())) ||
      (rc = dev_upload(h, &dmo, mp_off.data(), mp_off.size())) || (rc = dev_upload(h, &dm, mp.data(), mp.size())))
    return rc;
  A.n = n;
  A.spread_pair = spair; A.zsum = zsum; A.zread = zread; A.zone_key = t->zone_key; A.n_zone = n_zone;
  A.dom = dom; A.ident_sel = is; A.ident_anti = ia; A.ident_prio = ip;
  A.pair_sel = ps; A.pair_key = pk; A.pair_off = po; A.carry_key = ck; A.carry_off = co;
  A.ac = ac; A.terms = terms; A.carries = carries; A.cnt = cnt; A.carried = carried;
  A.mm = mm; A.part = part; A.ticket = ticket;
  A.aux_pair = apair; A.asum = asum; A.aread = aread; A.aux_w = t->aux_pair ? t->aux_weight : 0;
  A.aux_key = t->aux_pair ? t->aux_key : -1; A.aux_kind = t->aux_kind; A.n_adom = n_adom;
  A.svc_class = sv_cls; A.svc_miss = sv_miss; A.svc = sv; A.svc_conflict = sv_conf; A.svc_of_off = sv_of_off;
  A.svc_of = sv_of; A.n_svc = t->svc_class ? t->n_svc : 0; A.n_svc_labels = t->svc_class ? t->n_svc_labels : 0;
  A.n_pair = t->n_pair;
  A.sel_words = t->sel_words;
  A.carry_words = t->carry_words;
  KsimAff* dev;
  if ((rc = dev_upload(h, &dev, &A, 1))) return rc;
  HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  for (void* q : h->aff_bufs) dev_free(h, q);  // the previous tables (reload)
  h->aff_bufs.clear();
  for (size_t k = nb0; k < h->bufs.size(); ++k) h->aff_bufs.push_back(h->bufs[k].p);
  h->aff_dev = dev;
  h->aff_h = A;
  h->aff_ident_shared = ish;
  h->aff_aclass_shared = ash;
  h->aff_n_pair = t->n_pair;
  h->aff_n_carry = t->n_carry;
  h->aff_n_zone = n_zone;
  h->aff_n_keys = t->n_keys;
  h->pg_id_anti_off = dao; h->pg_id_anti = da; h->pg_id_prio_off = dpo; h->pg_id_prio = dp;
  h->pg_id_mp_off = dmo; h->pg_id_mp = dm;
  h->pg_max_anti = mx_anti; h->pg_max_prio = mx_prio; h->pg_max_mp = mx_mp;
  h->pg_max_req = mx_req; h->pg_max_pref = mx_pref; h->pg_max_car = mx_car;
  h->ctx.aff = dev;
  h->aff_n_ident = t->n_ident;
  h->aff_n_aclass = t->n_aclass;
  h->have_aff = true;
  h->aff_stale = false;
  // the table pointer is baked into the launch graph's kernel arguments
  if (h->gexec) { (void)hipGraphExecDestroy(h->gexec); h->gexec = nullptr; }
  if (h->graph) { (void)hipGraphDestroy(h->graph); h->graph = nullptr; }
  return KSIM_OK;
}
