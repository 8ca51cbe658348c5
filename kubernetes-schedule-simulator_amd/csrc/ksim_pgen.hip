// ksim_pgen.hip — the general persistent kernel for pods that carry inter-pod affinity terms,
// SelectorSpread selectors, volumes or a CheckServiceAffinity constraint,
// alongside every other supported pod: one launch walks the whole queue range, no per-pod launch.
//
// The per-pod cycle (core/generic_scheduler.go:112-198) of these pods needs two grid-wide
// reductions instead of one: InterPodAffinityPriority normalises over the min / max of the raw
// counts of the *fit* nodes (priorities/interpod_affinity.go:218-236) and SelectorSpread over the
// fit nodes' maximum count and per-zone sums (priorities/selector_spreading.go:121-174), and only
// then are the per-reduce-class maxima known.  Workgroup b owns the contiguous name-rank range
// [b*chunk, (b+1)*chunk); per pod:
//
//   1. every row: predicatesOrdering (pg_predicates, the ksim_predicates_a chain), map score, raw
//      InterPodAffinity sum, spread count;
//   2. pass A (pods that read either priority): the workgroup's (min, max, max count, haveZones,
//      zone sums) → one tagged record per workgroup; wave 0 sweeps every record;
//   3. the normalised scores are added; per reduce class (max, count) + fit count → tagged
//      granules; wave 0 sweeps them and decides (findNodesThatFit → NormalizeReduce →
//      selectHost's round-robin index, generic_scheduler.go:141-198), replicated in every
//      workgroup like lastNodeIndex;
//   4. the owner of the selected rank picks the row and commits it (NodeInfo.AddPod,
//      node_info.go:318-341: resource row, host ports, volume mounts, the affinity counts of its
//      row); a pod whose affinity counts live in shared topology domains (zones, "anywhere")
//      publishes the node in a tagged commit word and EVERY workgroup applies the counts to its
//      rows of that domain.
//
// Everything a row's evaluation and the commit touch is in LDS for the whole call: the resource
// row, label / taint set ids, the static (pod class, row) word, volume slots and per-filter mount
// counts, host-port slots, topology domains and the affinity counts in "row form" (for counted
// pair c and row j: the pair's count in j's domain of the pair's key, 0 without the key; carried
// terms likewise — every workgroup keeps its own rows, shared domains stay consistent by
// replication).  The pod's own data — descriptor, reduce-class values, affinity term lists,
// volume refs, zone verdicts, ports — is a contiguous record per pod (ksim_pgen_pack, before the
// launch); waves 1-3 load pod p+1's record while wave 0 is in pod p's exchange, so the cycle has
// no dependent global load.  HBM is written back at the end of the call (the canonical per-domain
// affinity counts through the rows' domains).
//
// The only cross-workgroup traffic is the tagged exchange (8-bit pod tag per 8-byte word, 4 slots
// by pod mod 4: a workgroup publishing pod p has read everyone's pod p-1 granules).  Every spin is
// bounded (2 s → error bit 4).
#include <algorithm>

#include "ksim_pgen.h"
#include "ksim_wave.h"

#define PG_BS 256
#define PG_NW (PG_BS / 64)
#define PG_NSLOT 4
#define PG_MAXG 256
#define PG_MAXZ 28
// words of a pass-A record: min, max, max count, haveZones, the spread zone sums, then the
// auxiliary priority's max count, summed count, haveZones and domain sums
#define PG_MAXAD 64  // the auxiliary priority's domains
#define PG_RA (4 + PG_MAXZ + 3 + PG_MAXAD)
#define PG_MAXL 256          // longest counted-pair / carry list of a pod (shared-domain commit)
// exchange buffer: pass-A records, class granules, then one commit word per slot
#define PG_COMMIT_OFF ((int64_t)PG_NSLOT * (PG_RA + KSIM_MAX_RCLASS) * PG_MAXG)
#define PG_GRAN_WORDS (PG_COMMIT_OFF + PG_NSLOT)
#define PG_LDS_BUDGET (154 * 1024)

// static (class, row) word
#define PG_ST_SEL 1u
#define PG_ST_TAINT 2u
#define PG_ST_NOEXEC 4u
#define PG_ST_SVC 0x1000u

namespace {

constexpr uint64_t M56 = (1ull << 56) - 1;
constexpr int64_t B55 = (int64_t)1 << 55;

__device__ __forceinline__ void pg_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t pg_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t* rec_at(uint64_t* g, int slot, int word, int b) {
  return g + ((int64_t)slot * PG_RA + word) * PG_MAXG + b;
}
__device__ __forceinline__ uint64_t* cls_at(uint64_t* g, int slot, int q, int b) {
  return g + (int64_t)PG_NSLOT * PG_RA * PG_MAXG + ((int64_t)slot * KSIM_MAX_RCLASS + q) * PG_MAXG + b;
}
__device__ __forceinline__ uint32_t gtag(uint64_t v) { return (uint32_t)(v >> 56); }
__device__ __forceinline__ int32_t gfit(uint64_t v) { return (int32_t)((v >> 44) & 0xFFF); }
__device__ __forceinline__ int32_t gcnt(uint64_t v) { return (int32_t)((v >> 32) & 0xFFF); }
__device__ __forceinline__ int32_t gscore(uint64_t v) { return (int32_t)(uint32_t)v; }

// The workgroup's LDS image (ksim_pgen_plan's layout).
struct PgL {
  int64_t *ac, *am, *rc, *rm, *zc, *zm;
  int32_t *al, *ct;
  uint32_t* fl;
  int32_t *ls, *ts, *sc;
  uint8_t* cl;
  uint16_t* st;
  int32_t* vc;
  uint16_t* vh;
  uint64_t* vs;
  int32_t* pc;
  uint64_t* pk;
  int32_t* dom;
  int32_t* cnt;
  int64_t* car;
  int32_t* hd;   // dense hypothesis deltas (null when not staged)
  int64_t* hc;
  int32_t* hk;
  int32_t* g0;   // [n_pair] domain-0 counts of every counted pair (the lender check's totals; null: off)
  int32_t chunk;
};

// The pod-context record in LDS: descriptor, header, section offsets.
struct PgX {
  const char* base;
  uint32_t so[PGS_END + 1];
  __device__ __forceinline__ const ksim_pod& pod() const { return *reinterpret_cast<const ksim_pod*>(base); }
  __device__ __forceinline__ const PgHdr& hdr() const { return *reinterpret_cast<const PgHdr*>(base + 128); }
  template <class T>
  __device__ __forceinline__ const T* sec(int s) const { return reinterpret_cast<const T*>(base + so[s]); }
  __device__ __forceinline__ int64_t tv(int q) const { return reinterpret_cast<const int64_t*>(base + 192)[q]; }
  __device__ __forceinline__ int64_t av(int q) const { return reinterpret_cast<const int64_t*>(base + 192)[KSIM_MAX_RCLASS + q]; }
  __device__ __forceinline__ int64_t ad(int q) const { return reinterpret_cast<const int64_t*>(base + 192)[2 * KSIM_MAX_RCLASS + q]; }
};

// The pod's uniform fields, read once from its LDS record into scalar registers (the evaluation's
// branches on them are then scalar, and no LDS round trip sits in front of them).
__device__ __forceinline__ int32_t rfl(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t rfl64(int64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ PgHdr pg_hdr_u(const PgHdr& x) {
  PgHdr h;
  h.K = rfl(x.K); h.k1 = rfl(x.k1); h.k2 = rfl(x.k2); h.sp = rfl(x.sp); h.fl = rfl(x.fl);
  h.n_anti = rfl(x.n_anti); h.n_req = rfl(x.n_req); h.n_pref = rfl(x.n_pref); h.n_prio = rfl(x.n_prio);
  h.n_mp = rfl(x.n_mp); h.n_car = rfl(x.n_car); h.n_ref = rfl(x.n_ref); h.vfilter = rfl(x.vfilter);
  h.n_zw = rfl(x.n_zw); h.n_port = rfl(x.n_port); h.n_scal = rfl(x.n_scal);
  return h;
}
// the fields the evaluation reads (the commit reads the record itself)
__device__ __forceinline__ ksim_pod pg_pod_u(const ksim_pod& x) {
  ksim_pod p{};
  p.req_cpu = rfl64(x.req_cpu); p.req_mem = rfl64(x.req_mem); p.req_gpu = rfl64(x.req_gpu); p.req_eph = rfl64(x.req_eph);
  p.nz_cpu = rfl64(x.nz_cpu); p.nz_mem = rfl64(x.nz_mem);
  p.cls = rfl(x.cls); p.host = rfl(x.host); p.flags = (uint32_t)rfl((int32_t)x.flags);
  p.scalar_off = rfl(x.scalar_off); p.scalar_cnt = rfl(x.scalar_cnt);
  p.aff_class = rfl(x.aff_class);  // (the lender check's affinity class)
  return p;
}

struct PgPref {
  int32_t pair, pad;
  int64_t weight;
};
struct PgCar {
  int32_t term, key;
  int64_t amount;
};

// Static word of (pod class, row) from the class tables (HBM): the staged form reads it from LDS.
__device__ __forceinline__ uint32_t pg_static_word(const KsimCtx& c, int32_t cls, int32_t ls, int32_t ts) {
  uint32_t w = 0;
  if (!ksim_bit(c.sel_ok, cls, c.lwords, ls)) w |= PG_ST_SEL;
  if (!ksim_bit(c.taint_ok, cls, c.twords, ts)) w |= PG_ST_TAINT;
  if (!ksim_bit(c.noexec_ok, cls, c.twords, ts)) w |= PG_ST_NOEXEC;
  w |= (uint32_t)(c.tt_class[(int64_t)cls * c.n_taint_sets + ts] & 15u) << 4;
  w |= (uint32_t)(c.na_class[(int64_t)cls * c.n_label_sets + ls] & 15u) << 8;
  if (c.svc_ok && !ksim_bit(c.svc_ok, cls, c.lwords, ls)) w |= PG_ST_SVC;
  return w;
}

// Volume slot s of row j (node i): the first vslots in LDS, the rest in HBM (authoritative there).
__device__ __forceinline__ uint64_t* pg_slot(const PGenArgs& g, const PgL& L, int32_t j, int64_t i, int32_t s) {
  return s < g.d.vslots ? &L.vs[(int64_t)s * L.chunk + j] : &g.V.slots[(int64_t)s * g.V.n + i];
}

__device__ __forceinline__ uint64_t pg_slot_get(const PGenArgs& g, const PgL& L, int32_t j, int64_t i, int32_t s) {
  return s < g.d.vslots ? L.vs[(int64_t)s * L.chunk + j] : g.V.slots[(int64_t)s * g.V.n + i];
}

__device__ __forceinline__ int32_t pg_vol_find(const PGenArgs& g, const PgL& L, int32_t j, int64_t i, int32_t cnt,
                                               int32_t key) {
  const int32_t cl = cnt < g.d.vslots ? cnt : g.d.vslots;
  for (int32_t s = 0; s < cl; ++s)
    if ((int32_t)(L.vs[(int64_t)s * L.chunk + j] >> 32) == key) return s;
  for (int32_t s = cl; s < cnt; ++s)
    if ((int32_t)(g.V.slots[(int64_t)s * g.V.n + i] >> 32) == key) return s;
  return -1;
}

// The previous pod p as a hypothesis on the evaluated row (the dual-hypothesis kernel): pod p+1
// is evaluated both on the row as it stands and as it would stand with p committed to it, so the
// owner of p's node needs no re-evaluation after the decision.  Only pods whose commit touches the
// row alone and the LDS image (no gpu / ephemeral / scalar requests, no shared-domain affinity
// counts) are hypotheses; the others take the re-evaluation path.
struct PgHyp {
  const PgX* X;    // pod p's record
  const PgHdr* H;  // its uniform header
};

__device__ __forceinline__ bool pg_port_hit(uint64_t wk, uint64_t e) {
  if ((e & 0xFFFFFFFFFFull) != (wk & 0xFFFFFFFFFFull)) return false;
  const uint32_t wip = (uint32_t)(wk >> 40), eip = (uint32_t)(e >> 40);
  return wip == 0 || eip == 0 || eip == wip;
}

// counted pair `pair` on row j (+1 when the hypothesis's identity matches it and j has its key)
template <bool HYP>
__device__ __forceinline__ int32_t pg_cnt(const PgL& L, const PgHyp& y, int32_t pair, int32_t j) {
  int32_t v = L.cnt[(int64_t)pair * L.chunk + j];
  if (HYP && L.hd) {  // the staged dense delta: one lookup
    const int32_t k1 = L.hd[pair];
    if (k1 && L.dom[(int64_t)(k1 - 1) * L.chunk + j] >= 0) v += 1;
  } else if (HYP) {
    const int2* mp = y.X->sec<int2>(PGS_MP);
    for (int32_t x = 0; x < y.H->n_mp; ++x)
      if (mp[x].x == pair && L.dom[(int64_t)mp[x].y * L.chunk + j] >= 0) v += 1;
  }
  return v;
}

// carried term e on row j (+ the hypothesis's carried amounts of e)
template <bool HYP>
__device__ __forceinline__ int64_t pg_car(const PgL& L, const PgHyp& y, int32_t e, int32_t j) {
  int64_t v = L.car[(int64_t)e * L.chunk + j];
  if (HYP && L.hk) {
    const int32_t k1 = L.hk[e];
    if (k1 && L.dom[(int64_t)(k1 - 1) * L.chunk + j] >= 0) v += L.hc[e];
  } else if (HYP) {
    const PgCar* cr = y.X->sec<PgCar>(PGS_CAR);
    for (int32_t x = 0; x < y.H->n_car; ++x)
      if (cr[x].term == e && L.dom[(int64_t)cr[x].key * L.chunk + j] >= 0) v += cr[x].amount;
  }
  return v;
}

// the hypothesis's mounts of volume key k: read-write / read-only inline mounts, any mount
template <bool HYP>
__device__ __forceinline__ void pg_hyp_mounts(const PgHyp& y, int32_t key, uint32_t* rw, uint32_t* ro, bool* any) {
  if (!HYP || !(y.H->fl & PGF_VOL)) return;
  const int4* r = y.X->sec<int4>(PGS_REF);
  for (int32_t x = 0; x < y.H->n_ref; ++x) {
    if (r[x].x != key) continue;
    const uint32_t f = (uint32_t)r[x].y;
    *any = true;
    if (f & KSIM_VOL_VIA_PVC) continue;
    if (f & KSIM_VOL_READ_ONLY) *ro += 1;
    else *rw += 1;
  }
}

// CheckServiceAffinity's labels from the lender (ksim_svc_lender, predicates.go:986-1011) on row j:
// the totals (key 0, every node in domain 0) and the label-presence counts from the workgroup's
// domain-0 copies (L.g0), the count in j's domain of the label value's key from the row form.
__device__ __forceinline__ uint32_t pg_svc_lender(const KsimCtx& c, const PGenArgs& g, const PgL& L, int32_t a, int32_t j) {
  const KsimAff& A = g.A;
  const int32_t v = A.svc_class[a];
  if (v < 0) return 0;
  const uint32_t miss = A.svc_miss[a];
  const ksim_svc_ident& S = A.svc[v];
  const int32_t total = L.g0[S.pair_all];
  if (total == 0) return 0;  // no cached pod to lend labels
  if (__hip_atomic_load(&A.svc_conflict[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & miss) {
    atomicOr(c.err, 128);
    return 1u << KSIM_R_SERVICE_AFFINITY;
  }
  for (uint32_t mm = miss; mm; mm &= mm - 1) {
    const int l = __builtin_ctz(mm);
    if (L.g0[S.pair_present[l]] == 0) continue;  // the lender lacks l: no constraint
    const int32_t pv = S.pair_value[l];
    if (L.dom[(int64_t)A.pair_key[pv] * L.chunk + j] < 0 || L.cnt[(int64_t)pv * L.chunk + j] != total)
      return 1u << KSIM_R_SERVICE_AFFINITY;
  }
  return 0;
}

// ksim_svc_commit on row j before the commit of an identity's pod adds its counts: the
// service-affinity identities it matches record the labels on which the row disagrees with their
// earlier cached pods.  One thread.
__device__ __forceinline__ void pg_svc_commit(const PGenArgs& g, const PgL& L, int32_t ident, int32_t j) {
  const KsimAff& A = g.A;
  for (int32_t e = A.svc_of_off[ident - 1], end = A.svc_of_off[ident]; e < end; ++e) {
    const int32_t v = A.svc_of[e];
    const ksim_svc_ident& S = A.svc[v];
    const int32_t total = L.g0[S.pair_all];
    if (total == 0) continue;  // the first one: nothing to disagree with
    uint32_t bad = 0;
    for (int l = 0; l < A.n_svc_labels; ++l) {
      const int32_t pv = S.pair_value[l];
      const int32_t d = L.dom[(int64_t)A.pair_key[pv] * L.chunk + j];
      const int32_t here = d >= 0 ? L.cnt[(int64_t)pv * L.chunk + j] : total - L.g0[S.pair_present[l]];
      if (here != total) bad |= 1u << l;
    }
    if (bad) atomicOr(&A.svc_conflict[v], bad);
  }
}

// The first failing predicate of predicatesOrdering (predicates.go:129-138) on row j (node i),
// exactly the chain of ksim_predicates_a, over the LDS image and the pod's record (HYP: with the
// hypothesis pod committed to the row: r carries its resources).  0 = fits.
template <bool HYP>
__device__ __forceinline__ uint32_t pg_predicates(const KsimCtx& c, const PGenArgs& g, const PgL& L, const PgX& X,
                                                  const ksim_pod& P, const PgHdr& H, int32_t j, int64_t i,
                                                  const KsimRow& r, uint32_t st, const PgHyp& y, uint64_t* sa = nullptr) {
  const uint32_t pr = c.preds;
  uint32_t m;
#ifdef KSIM_STAMPS
  uint64_t ts_ = __builtin_amdgcn_s_memtime();
#define EV_T(k)                                          \
  do {                                                   \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();   \
    if (sa) sa[k] += t_ - ts_;                           \
    ts_ = t_;                                            \
  } while (0)
#else
#define EV_T(k) \
  do {          \
  } while (0)
#endif
  if (pr & KSIM_P_CHECK_NODE_CONDITION) {
    m = r.fl & KSIM_COND_REASON_MASK;  // bit positions coincide with KSIM_R_*
    if (m) return m;
  }
  if ((pr & KSIM_P_CHECK_NODE_UNSCHEDULABLE) && (r.fl & KSIM_N_UNSCHEDULABLE)) return 1u << KSIM_R_UNSCHEDULABLE;
  const uint32_t sel = ((P.flags & KSIM_POD_NEED_SELECTOR) && (st & PG_ST_SEL)) ? (1u << KSIM_R_NODE_SELECTOR) : 0u;
  // HostPortInfo.CheckConflict (pkg/scheduler/util/utils.go:101-130) over the row's LDS slots
  uint32_t ports = 0;
  if (H.n_port && (pr & (KSIM_P_GENERAL | KSIM_P_HOST_PORTS))) {
    const uint64_t* want = X.sec<uint64_t>(PGS_PORT);
    const int32_t pcn = g.d.pslots ? L.pc[j] : 0;
    for (int32_t k = 0; k < H.n_port && !ports; ++k) {
      const uint64_t wk = want[k];
      for (int32_t s = 0; s < pcn; ++s)
        if (pg_port_hit(wk, L.pk[(int64_t)s * L.chunk + j])) { ports = 1u << KSIM_R_HOST_PORTS; break; }
      if (HYP && !ports) {
        const uint64_t* hp = y.X->sec<uint64_t>(PGS_PORT);
        for (int32_t s = 0; s < y.H->n_port; ++s)
          if (pg_port_hit(wk, hp[s])) { ports = 1u << KSIM_R_HOST_PORTS; break; }
      }
    }
  }
  if (pr & KSIM_P_GENERAL) {
    m = ksim_resources(c, P, i, r) | ksim_hostname(P, i) | sel | ports;
    if (m) return m;
  }
  if (pr & KSIM_P_HOSTNAME) {
    m = ksim_hostname(P, i);
    if (m) return m;
  }
  if ((pr & KSIM_P_HOST_PORTS) && ports) return ports;
  if ((pr & KSIM_P_NODE_SELECTOR) && sel) return sel;
  if (pr & KSIM_P_RESOURCES) {
    m = ksim_resources(c, P, i, r);
    if (m) return m;
  }
  EV_T(1);
  const bool vol = (H.fl & PGF_VOL) != 0;
  const int4* refs = X.sec<int4>(PGS_REF);
  const int32_t vcn = (vol && g.d.vcap) ? L.vc[j] : 0;
  if ((pr & KSIM_P_DISK_CONFLICT) && vol && (vcn || (HYP && (y.H->fl & PGF_VOL)))) {
    // NoDiskConflict (predicates.go:276-285 over isVolumeConflict :220-265)
    for (int32_t x = 0; x < H.n_ref; ++x) {
      const int4 ref = refs[x];
      const uint32_t f = (uint32_t)ref.y;
      if (!(f & (KSIM_VOL_CONFLICT_ANY | KSIM_VOL_CONFLICT_RW))) continue;
      const int32_t s = pg_vol_find(g, L, j, i, vcn, ref.x);
      uint32_t rw = 0, ro = 0;
      bool any = false;
      if (s >= 0) {
        const uint64_t w = pg_slot_get(g, L, j, i, s);
        rw = (uint32_t)(w & 0x7FFu);
        ro = (uint32_t)((w >> 11) & 0x7FFu);
      }
      pg_hyp_mounts<HYP>(y, ref.x, &rw, &ro, &any);
      if ((f & KSIM_VOL_CONFLICT_ANY) ? (rw + ro > 0) : (rw > 0)) return 1u << KSIM_R_DISK_CONFLICT;
    }
  }
  EV_T(2);
  if ((pr & KSIM_P_TAINTS) && (P.flags & KSIM_POD_NEED_TAINTS) && (st & PG_ST_TAINT)) return 1u << KSIM_R_TAINTS;
  if ((pr & KSIM_P_NOEXEC_TAINTS) && (P.flags & KSIM_POD_NEED_TAINTS) && (st & PG_ST_NOEXEC)) return 1u << KSIM_R_TAINTS;
  if ((pr & KSIM_P_LABEL_PRESENCE) && (r.fl & KSIM_N_LABEL_PRESENCE)) return 1u << KSIM_R_LABEL_PRESENCE;
  if ((pr & KSIM_P_SERVICE_AFFINITY) && (P.flags & KSIM_POD_NEED_SVC_AFFINITY) && (st & PG_ST_SVC))
    return 1u << KSIM_R_SERVICE_AFFINITY;
  if (!HYP && L.g0 && (pr & KSIM_P_SERVICE_AFFINITY) && P.aff_class > 0) {
    m = pg_svc_lender(c, g, L, P.aff_class - 1, j);
    if (m) return m;
  }
  if (vol) {
    // MaxEBS / MaxGCEPD / MaxAzureDiskVolumeCount (predicates.go:415-456): the row's mounted keys
    // each filter counts (LDS) plus the pod's new keys not mounted yet
    const uint32_t which = ((pr & KSIM_P_MAX_EBS) ? KSIM_VOL_EBS : 0u) | ((pr & KSIM_P_MAX_GCE_PD) ? KSIM_VOL_GCE_PD : 0u) |
                           ((pr & KSIM_P_MAX_AZURE_DISK) ? KSIM_VOL_AZURE_DISK : 0u);
    const uint32_t want = (uint32_t)H.vfilter & which;
    if (want) {
      for (int t = 0; t < 3; ++t) {
        const uint32_t f = 1u << t;
        if (!(want & f)) continue;
        int32_t add = 0;
        for (int32_t x = 0; x < H.n_ref; ++x) {
          const int4 ref = refs[x];
          if (!(((uint32_t)ref.y & KSIM_VOL_NEW) && ((uint32_t)ref.z & f)) || pg_vol_find(g, L, j, i, vcn, ref.x) >= 0) continue;
          uint32_t rw = 0, ro = 0;
          bool any = false;
          pg_hyp_mounts<HYP>(y, ref.x, &rw, &ro, &any);
          if (!any) ++add;
        }
        int32_t have = g.d.vcap ? (int32_t)L.vh[(int64_t)t * L.chunk + j] : 0;
        if (HYP && (y.H->fl & PGF_VOL)) {  // the hypothesis's keys this filter counts, not mounted yet
          const int4* hr = y.X->sec<int4>(PGS_REF);
          for (int32_t x = 0; x < y.H->n_ref; ++x)
            if (((uint32_t)hr[x].y & KSIM_VOL_NEW) && ((uint32_t)hr[x].z & f) && pg_vol_find(g, L, j, i, vcn, hr[x].x) < 0) ++have;
        }
        if (have + add > g.V.max_vols[t]) return 1u << KSIM_R_MAX_VOLUME_COUNT;
      }
    }
    // NoVolumeZoneConflict (predicates.go:539-633): a (volume class, label set) verdict
    if ((pr & KSIM_P_VOLUME_ZONE) && H.n_zw) {
      const int32_t ls = L.ls[j];
      if (!((X.sec<uint32_t>(PGS_ZOK)[ls >> 5] >> (ls & 31)) & 1u)) return 1u << KSIM_R_VOLUME_ZONE;
    }
  }
  EV_T(3);
  if ((pr & KSIM_P_MEM_PRESSURE) && (P.flags & KSIM_POD_BEST_EFFORT) && (r.fl & KSIM_N_MEM_PRESSURE))
    return 1u << KSIM_R_MEM_PRESSURE;
  if ((pr & KSIM_P_DISK_PRESSURE) && (r.fl & KSIM_N_DISK_PRESSURE)) return 1u << KSIM_R_DISK_PRESSURE;
  if ((pr & KSIM_P_INTERPOD_AFFINITY) && (H.fl & PGF_AFF)) {
    // MatchInterPodAffinity (predicates.go:1143-1450) over the row-form counts: existing pods'
    // required anti-affinity terms the pod matches (satisfiesExistingPodsAntiAffinity
    // :1340-1379), then its own required affinity terms (a term no placed pod matches is waived
    // when the pod matches it itself, :1405-1424) and required anti-affinity terms (:1430-1441)
    const uint32_t base = 1u << KSIM_R_POD_AFFINITY;
    const int32_t* anti = X.sec<int32_t>(PGS_ANTI);
    for (int32_t x = 0; x < H.n_anti; ++x)
      if (pg_car<HYP>(L, y, anti[x], j) > 0) return base | (1u << KSIM_R_EXISTING_ANTI_AFFINITY);
    const int4* req = X.sec<int4>(PGS_REQ);
    for (int32_t x = 0; x < H.n_req; ++x) {
      const int4 t = req[x];
      const bool match = L.dom[(int64_t)t.y * L.chunk + j] >= 0 && pg_cnt<HYP>(L, y, t.x, j) > 0;
      if ((t.w & 0xFF) == KSIM_AFF_REQ_AFFINITY) {
        if (!match && (!(t.w >> 8) || pg_cnt<HYP>(L, y, t.z, j) > 0)) return base | (1u << KSIM_R_AFFINITY_RULES);
      } else if (match) {
        return base | (1u << KSIM_R_ANTI_AFFINITY_RULES);
      }
    }
  }
  EV_T(4);
  return 0;
}
#undef EV_T

// CalculateInterPodAffinityPriority's per-node sum (interpod_affinity.go:124-214) before the
// normalisation, over the row-form counts (0 on rows without the term's key, as in Go).
template <bool HYP>
__device__ __forceinline__ int64_t pg_interpod_raw(const PgL& L, const PgX& X, const PgHdr& H, int32_t j, const PgHyp& y) {
  int64_t s = 0;
  const PgPref* pref = X.sec<PgPref>(PGS_PREF);
  for (int32_t x = 0; x < H.n_pref; ++x) s += pref[x].weight * (int64_t)pg_cnt<HYP>(L, y, pref[x].pair, j);
  const int32_t* prio = X.sec<int32_t>(PGS_PRIO);
  for (int32_t x = 0; x < H.n_prio; ++x) s += pg_car<HYP>(L, y, prio[x], j);
  return s;
}

// The workgroup's LDS image from the planned offsets.
__device__ __forceinline__ PgL pg_lds(char* sm, const PGenArgs& g, int64_t chunk) {
  PgL L;
  L.chunk = (int32_t)chunk;
  L.ac = (int64_t*)(sm + g.off[PGO_AC]); L.am = (int64_t*)(sm + g.off[PGO_AM]);
  L.rc = (int64_t*)(sm + g.off[PGO_RC]); L.rm = (int64_t*)(sm + g.off[PGO_RM]);
  L.zc = (int64_t*)(sm + g.off[PGO_ZC]); L.zm = (int64_t*)(sm + g.off[PGO_ZM]);
  L.al = (int32_t*)(sm + g.off[PGO_AL]); L.ct = (int32_t*)(sm + g.off[PGO_CT]);
  L.fl = (uint32_t*)(sm + g.off[PGO_FL]); L.ls = (int32_t*)(sm + g.off[PGO_LS]);
  L.ts = (int32_t*)(sm + g.off[PGO_TS]); L.sc = (int32_t*)(sm + g.off[PGO_SC]);
  L.cl = (uint8_t*)(sm + g.off[PGO_CL]); L.st = (uint16_t*)(sm + g.off[PGO_ST]);
  L.vc = (int32_t*)(sm + g.off[PGO_VC]); L.vh = (uint16_t*)(sm + g.off[PGO_VH]);
  L.vs = (uint64_t*)(sm + g.off[PGO_VS]); L.pc = (int32_t*)(sm + g.off[PGO_PC]);
  L.pk = (uint64_t*)(sm + g.off[PGO_PK]); L.dom = (int32_t*)(sm + g.off[PGO_DOM]);
  L.cnt = (int32_t*)(sm + g.off[PGO_CNT]); L.car = (int64_t*)(sm + g.off[PGO_CAR]);
  L.hd = g.d.hdense ? (int32_t*)(sm + g.off[PGO_HD]) : nullptr;
  L.hc = g.d.hdense ? (int64_t*)(sm + g.off[PGO_HC]) : nullptr;
  L.hk = g.d.hdense ? (int32_t*)(sm + g.off[PGO_HK]) : nullptr;
  L.g0 = nullptr;
  return L;
}
// pod-context record r & 1 (offset arithmetic on the LDS base keeps the accesses ds_*)
__device__ __forceinline__ char* pg_xrec(char* sm, const PGenArgs& g, int64_t r) {
  return sm + g.off[PGO_X0] + (uint32_t)(r & 1) * (g.off[PGO_X1] - g.off[PGO_X0]);
}

}  // namespace


// ---- staging and write-back shared by both persistent forms ----
__device__ __forceinline__ void pg_stage_rows(const KsimCtx& c, const PGenArgs& g, const PgL& L, int64_t lo, int32_t nrows,
                                              int64_t chunk, int tid, int nthr) {
  const int64_t n = c.n;
  const int32_t vsl = g.d.vslots, vcap = g.d.vcap, psl = g.d.pslots;
  for (int32_t j = tid; j < nrows; j += nthr) {
    const int64_t i = lo + j;
    L.ac[j] = c.alloc_cpu[i]; L.am[j] = c.alloc_mem[i];
    L.rc[j] = c.req_cpu[i]; L.rm[j] = c.req_mem[i]; L.zc[j] = c.nz_cpu[i]; L.zm[j] = c.nz_mem[i];
    L.al[j] = c.allowed_pods[i]; L.ct[j] = c.pod_count[i]; L.fl[j] = c.flags[i];
    L.ls[j] = c.label_set[i]; L.ts[j] = c.taint_set[i];
    if (psl) {
      const int32_t pc = c.port_count[i];
      L.pc[j] = pc;
      for (int32_t s = 0; s < pc; ++s) L.pk[(int64_t)s * chunk + j] = c.ports[(int64_t)s * n + i];
    }
    if (vcap) {
      const int32_t vc = g.V.slot_count[i];
      L.vc[j] = vc;
      uint32_t h0 = 0, h1 = 0, h2 = 0;
      for (int32_t s = 0; s < vc; ++s) {
        const uint64_t w = g.V.slots[(int64_t)s * n + i];
        if (s < vsl) L.vs[(int64_t)s * chunk + j] = w;
        const uint32_t f = g.V.key_filter[(int32_t)(w >> 32)];
        h0 += f & 1u; h1 += (f >> 1) & 1u; h2 += (f >> 2) & 1u;
      }
      L.vh[j] = (uint16_t)h0; L.vh[chunk + j] = (uint16_t)h1; L.vh[2 * chunk + j] = (uint16_t)h2;
    }
  }
  for (int32_t x = tid; x < g.d.n_keys * nrows; x += nthr) {
    const int32_t k = x / nrows, j = x - k * nrows;
    L.dom[(int64_t)k * chunk + j] = g.A.dom[(int64_t)k * n + lo + j];
  }
}

__device__ __forceinline__ void pg_stage_counts(const KsimCtx& c, const PGenArgs& g, const PgL& L, int32_t nrows,
                                                int64_t chunk, int tid, int nthr) {
  // affinity counts in row form, from the canonical per-domain counts
  for (int32_t x = tid; x < g.d.n_pair * nrows; x += nthr) {
    const int32_t cp = x / nrows, j = x - cp * nrows;
    const int32_t d = L.dom[(int64_t)g.A.pair_key[cp] * chunk + j];
    L.cnt[(int64_t)cp * chunk + j] = d >= 0 ? g.A.cnt[g.A.pair_off[cp] + d] : 0;
  }
  for (int32_t x = tid; x < g.d.n_carry * nrows; x += nthr) {
    const int32_t e = x / nrows, j = x - e * nrows;
    const int32_t d = L.dom[(int64_t)g.A.carry_key[e] * chunk + j];
    L.car[(int64_t)e * chunk + j] = d >= 0 ? g.A.carried[g.A.carry_off[e] + d] : 0;
  }
  if (g.d.n_st)  // static (pod class, row) words from the class tables
    for (int32_t k = tid; k < g.d.n_st * nrows; k += nthr) {
      const int32_t cls = k / nrows, j = k - cls * nrows;
      L.st[(int64_t)cls * chunk + j] = (uint16_t)pg_static_word(c, cls, L.ls[j], L.ts[j]);
    }
}

__device__ __forceinline__ void pg_write_back(const KsimCtx& c, const PGenArgs& g, const PgL& L, int64_t lo, int32_t nrows,
                                              int64_t chunk, int tid, int nthr) {
  const int64_t n = c.n;
  const int32_t vsl = g.d.vslots, vcap = g.d.vcap, psl = g.d.pslots;
  __syncthreads();
  for (int32_t j = tid; j < nrows; j += nthr) {
    const int64_t i = lo + j;
    c.req_cpu[i] = L.rc[j]; c.req_mem[i] = L.rm[j]; c.nz_cpu[i] = L.zc[j]; c.nz_mem[i] = L.zm[j];
    c.pod_count[i] = L.ct[j]; c.flags[i] = L.fl[j];
    if (psl) {
      const int32_t pc = L.pc[j];
      c.port_count[i] = pc;
      for (int32_t s = 0; s < pc; ++s) c.ports[(int64_t)s * n + i] = L.pk[(int64_t)s * chunk + j];
    }
    if (vcap) {
      const int32_t vc = L.vc[j];
      g.V.slot_count[i] = vc;
      for (int32_t s = 0; s < vc && s < vsl; ++s) g.V.slots[(int64_t)s * n + i] = L.vs[(int64_t)s * chunk + j];
    }
  }
  // canonical per-domain counts: every row of a domain holds the same value, so concurrent
  // identical stores from several workgroups are benign
  for (int32_t x = tid; x < g.d.n_pair * nrows; x += nthr) {
    const int32_t cp = x / nrows, j = x - cp * nrows;
    const int32_t d = L.dom[(int64_t)g.A.pair_key[cp] * chunk + j];
    if (d >= 0) g.A.cnt[g.A.pair_off[cp] + d] = L.cnt[(int64_t)cp * chunk + j];
  }
  for (int32_t x = tid; x < g.d.n_carry * nrows; x += nthr) {
    const int32_t e = x / nrows, j = x - e * nrows;
    const int32_t d = L.dom[(int64_t)g.A.carry_key[e] * chunk + j];
    if (d >= 0) g.A.carried[g.A.carry_off[e] + d] = L.car[(int64_t)e * chunk + j];
  }
}

#ifdef KSIM_STAMPS
// per-phase cycle sums of workgroup 0's thread 0 (s_memtime), written to c.dbg at the end
#define PG_STAMP(k)                                    \
  do {                                                 \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += t_ - t_prev;                         \
    t_prev = t_;                                      \
  } while (0)
#else
#define PG_STAMP(k) \
  do {              \
  } while (0)
#endif

// ---- ksim_pgen_pack: one pod-context record per queued pod of [first, end) ----
__global__ __launch_bounds__(64) void ksim_pgen_pack_kernel(KsimCtx c, PGenArgs g) {
  const int lane = threadIdx.x;
  const int64_t count = c.end - c.first;
  for (int64_t q = blockIdx.x; q < count; q += gridDim.x) {
    const int64_t pod = c.first + q;
    char* R = g.rec + q * (int64_t)g.d.rec_stride;
    const ksim_pod P = c.pods[pod];
    if (lane < 32) reinterpret_cast<uint32_t*>(R)[lane] = reinterpret_cast<const uint32_t*>(c.pods + pod)[lane];
    PgHdr H{};
    H.k1 = (c.w[KSIM_W_TAINT_TOLERATION] != 0) ? c.n_tt[P.cls] : 1;
    H.k2 = c.use_na ? c.n_na[P.cls] : 1;
    H.K = H.k1 * H.k2;
    const bool aff = g.has_aff && (P.aff_ident > 0 || P.aff_class > 0);
    const int32_t* ac = (aff && P.aff_class > 0) ? g.A.ac + 6 * (int64_t)(P.aff_class - 1) : nullptr;
    H.sp = (g.has_aff && !c.no_prio && c.w[KSIM_W_SELECTOR_SPREAD] != 0) ? ksim_spread_pair(g.A, P) : -1;
    if (g.has_aff && !c.no_prio && g.A.aux_pair && g.A.aux_w != 0) {  // (ipa_norm's aon / ap)
      const int32_t ap = ksim_aux_pair(g.A, P);
      if (ap >= 0 || g.A.aux_kind == KSIM_AUX_SERVICE_ANTI) H.fl |= PGF_AUX | ((ap + 1) << PGF_AUX_SHIFT);
    }
    int32_t a0 = 0, p0 = 0, m0 = 0;
    if (aff && P.aff_ident > 0) {
      const int32_t id = P.aff_ident - 1;
      a0 = g.id_anti_off[id]; H.n_anti = g.id_anti_off[id + 1] - a0;
      p0 = g.id_prio_off[id]; H.n_prio = g.id_prio_off[id + 1] - p0;
      m0 = g.id_mp_off[id];   H.n_mp = g.id_mp_off[id + 1] - m0;
    }
    if (ac) { H.n_req = ac[1]; H.n_pref = ac[3]; H.n_car = ac[5]; }
    if (aff) {
      H.fl |= PGF_AFF;
      if (!c.no_prio && c.w[KSIM_W_INTERPOD_AFFINITY] != 0 && (H.n_pref > 0 || H.n_prio > 0)) H.fl |= PGF_IPA;
      if (!c.no_commit && ((P.aff_ident > 0 && g.ident_shared[P.aff_ident - 1]) ||
                           (P.aff_class > 0 && g.aclass_shared[P.aff_class - 1])))
        H.fl |= PGF_SHARED;
      // a lender (its identity matches a service-affinity selector): every workgroup follows its
      // commit, for the domain-0 copies of the lender check's totals (even on node-like keys)
      if (!c.no_commit && g.svc_on && P.aff_ident > 0 && g.A.svc_of_off[P.aff_ident - 1] < g.A.svc_of_off[P.aff_ident])
        H.fl |= PGF_SHARED;
    }
    const int32_t* vc = nullptr;
    if (g.has_vol && P.vol_class > 0) {
      H.fl |= PGF_VOL;
      vc = g.V.vc + 2 * (int64_t)(P.vol_class - 1);
      H.n_ref = vc[1];
      H.vfilter = (int32_t)g.V.vc_filter[P.vol_class - 1];
      H.n_zw = (g.V.zone_ok && (c.preds & KSIM_P_VOLUME_ZONE)) ? g.V.zone_words : 0;
    }
    H.n_port = P.port_cnt;
    H.n_scal = P.scalar_cnt;
    if ((H.fl & PGF_SHARED) || P.add_gpu || P.add_eph || H.n_scal) H.fl |= PGF_NOHYP;
    uint32_t so[PGS_END + 1];
    pg_sections(H, so);
    if (so[PGS_END] > (uint32_t)g.d.rec_stride) {  // the host's bound is wrong: never write past the record
      if (lane == 0) atomicOr(c.err, 2);
      continue;
    }
    if (lane == 0) *reinterpret_cast<PgHdr*>(R + 128) = H;
    if (lane < KSIM_MAX_RCLASS) {
      int64_t* v = reinterpret_cast<int64_t*>(R + 192);
      v[lane] = c.tt_val[(int64_t)P.cls * c.val_w + lane];
      v[KSIM_MAX_RCLASS + lane] = c.na_val[(int64_t)P.cls * c.val_w + lane];
      v[2 * KSIM_MAX_RCLASS + lane] = c.na_add ? c.na_add[(int64_t)P.cls * c.val_w + lane] : 0;
    }
    for (int32_t x = lane; x < H.n_anti; x += 64) reinterpret_cast<int32_t*>(R + so[PGS_ANTI])[x] = g.id_anti[a0 + x];
    for (int32_t x = lane; x < H.n_prio; x += 64) reinterpret_cast<int32_t*>(R + so[PGS_PRIO])[x] = g.id_prio[p0 + x];
    for (int32_t x = lane; x < H.n_req; x += 64) {
      const ksim_aff_term t = g.A.terms[ac[0] + x];
      reinterpret_cast<int4*>(R + so[PGS_REQ])[x] = make_int4(t.pair, t.gate_key, t.exist_pair, t.kind | (t.self_ok ? 256 : 0));
    }
    for (int32_t x = lane; x < H.n_pref; x += 64) {
      const ksim_aff_term t = g.A.terms[ac[2] + x];
      PgPref& o = reinterpret_cast<PgPref*>(R + so[PGS_PREF])[x];
      o.pair = t.pair; o.pad = 0; o.weight = t.weight;
    }
    for (int32_t x = lane; x < H.n_mp; x += 64)
      reinterpret_cast<int2*>(R + so[PGS_MP])[x] = make_int2(g.id_mp[2 * (m0 + x)], g.id_mp[2 * (m0 + x) + 1]);
    for (int32_t x = lane; x < H.n_car; x += 64) {
      const ksim_aff_carry k = g.A.carries[ac[4] + x];
      PgCar& o = reinterpret_cast<PgCar*>(R + so[PGS_CAR])[x];
      o.term = k.term; o.key = g.A.carry_key[k.term]; o.amount = k.amount;
    }
    for (int32_t x = lane; x < H.n_ref; x += 64) {
      const ksim_vol_ref r = g.V.refs[vc[0] + x];
      reinterpret_cast<int4*>(R + so[PGS_REF])[x] = make_int4(r.key, (int32_t)r.flags, (int32_t)g.V.key_filter[r.key], 0);
    }
    for (int32_t x = lane; x < H.n_zw; x += 64)
      reinterpret_cast<uint32_t*>(R + so[PGS_ZOK])[x] = g.V.zone_ok[(int64_t)(P.vol_class - 1) * g.V.zone_words + x];
    for (int32_t x = lane; x < H.n_port; x += 64) reinterpret_cast<uint64_t*>(R + so[PGS_PORT])[x] = c.pod_ports[P.port_off + x];
    for (int32_t x = lane; x < H.n_scal; x += 64)
      reinterpret_cast<ksim_scalar_req*>(R + so[PGS_SCAL])[x] = c.pod_scalars[P.scalar_off + x];
  }
}

template <int NPT, int MB>
__global__ __launch_bounds__(PG_BS) void ksim_pgen_kernel(KsimCtx c_arg, PGenArgs g_arg) {
  extern __shared__ __attribute__((aligned(16))) char pg_smem[];
  __shared__ int64_t s_a[7][PG_NW];                  // pass A per wave: min, max, max count, haveZones, aux max / sum / haveZones
  __shared__ unsigned long long s_z[PG_MAXZ];        // pass A zone sums of this workgroup
  __shared__ unsigned long long s_az[PG_MAXAD];      // the auxiliary priority's domain sums of this workgroup
  __shared__ int64_t s_g[9];                         // pass A over the grid: min, max, max count, haveZones, max zone,
                                                     // aux max count, summed count, haveZones, max domain sum
  __shared__ int64_t s_gz[PG_MAXZ];                  // countsByZone over the grid
  __shared__ int64_t s_gaz[PG_MAXAD];                // the auxiliary domain sums over the grid
  __shared__ int32_t s_mx[PG_NW][KSIM_MAX_RCLASS];   // class partials per wave
  __shared__ int32_t s_cn[PG_NW][KSIM_MAX_RCLASS];
  __shared__ int32_t s_fit[PG_NW];
  __shared__ int32_t s_mode, s_blk, s_rank, s_abort;
  __shared__ uint32_t s_win;
  __shared__ int32_t s_tgt[KSIM_MAX_RCLASS];         // winning class q: its maximum (else -2)
  __shared__ int64_t s_node;
  __shared__ int32_t s_dw[PG_MAXL * 2];              // shared-domain commit: the node's domain per list entry
  __shared__ uint64_t s_bal[NPT][PG_NW];             // owner: each wave's ballot of its rows at the chosen score
  __shared__ int32_t s_g0[PG_SVC_PAIRS];             // the lender check: domain-0 counts of the counted pairs
#ifdef KSIM_STAMPS
  uint64_t st_acc[16] = {};
  uint64_t t_prev = __builtin_amdgcn_s_memtime();
#endif

  const KsimCtx& c = c_arg;
  const PGenArgs& g = g_arg;
  if (g.test_stall && blockIdx.x == gridDim.x - 1) return;  // diagnostic: a workgroup that never ran
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int G = gridDim.x;
  const int64_t chunk = c.chunk;
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = (lo + chunk < c.n) ? lo + chunk : c.n;
  const int32_t nrows = (int32_t)(hi - lo);
  const int64_t n = c.n;
  PgL L = pg_lds(pg_smem, g, chunk);
  if (g.svc_on) {  // (n_pair <= PG_SVC_PAIRS, host-checked)
    L.g0 = s_g0;
    for (int32_t cp = threadIdx.x; cp < g.d.n_pair; cp += PG_BS) s_g0[cp] = g.A.cnt[g.A.pair_off[cp]];
  }
  auto xrec = [&](int64_t r) { return pg_xrec(pg_smem, g, r); };
  const int32_t vcap = g.d.vcap, psl = g.d.pslots;

  pg_stage_rows(c, g, L, lo, nrows, chunk, tid, blockDim.x);
  // the pod-context record of the first pod
  {
    const uint4* src = reinterpret_cast<const uint4*>(g.rec);
    uint4* dst = reinterpret_cast<uint4*>(xrec(c.first));
    for (int32_t x = tid; x < g.d.rec_stride / 16; x += PG_BS) dst[x] = src[x];
  }
  if (tid == 0) s_abort = 0;
  if (tid < PG_MAXZ) s_z[tid] = 0;
  if (tid < PG_MAXAD) s_az[tid] = 0;
  uint64_t counter = *c.counter;  // replicated genericScheduler.lastNodeIndex (wave 0)
  __syncthreads();
  pg_stage_counts(c, g, L, nrows, chunk, tid, blockDim.x);
  __syncthreads();

  int64_t stop_pod = c.end;  // first pod not scheduled (a spin bound ran out: the grid is not co-resident)
  for (int64_t pod = c.first; pod < c.end; ++pod) {
    PgX X;
    X.base = xrec(pod);
    const PgHdr H = pg_hdr_u(X.hdr());
    pg_sections(H, X.so);
    const ksim_pod P = pg_pod_u(X.pod());
    const int K = H.K, k1 = H.k1, k2 = H.k2;
    const bool ipa = (H.fl & PGF_IPA) != 0;
    const int32_t sp = H.sp;
    const bool aon = (H.fl & PGF_AUX) != 0;
    const int32_t ap = (H.fl >> PGF_AUX_SHIFT) - 1;  // (-1 without PGF_AUX too)
    const uint32_t tag = (uint32_t)((pod - c.first + 1) & 0xFF);
    const int slot = (int)(pod % PG_NSLOT);
    // waves 1-3: pod p+1's record, loaded now and stored into the other LDS record during the
    // exchange (the buffer held pod p-1's, which every wave has finished with)
    const bool pf = wv > 0 && pod + 1 < c.end;
    const int32_t pfw = g.d.rec_stride / 16;
    uint4 pf0 = make_uint4(0, 0, 0, 0), pf1 = make_uint4(0, 0, 0, 0);
    if (pf) {
      const uint4* src = reinterpret_cast<const uint4*>(g.rec + (pod + 1 - c.first) * (int64_t)g.d.rec_stride);
      const int t = tid - 64;
      if (t < pfw) pf0 = src[t];
      if (t + 3 * 64 < pfw) pf1 = src[t + 3 * 64];
    }

    // ---- 1. evaluate this workgroup's rows ----
    bool fit[NPT];
    int64_t sc[NPT], raw[NPT], cnt[NPT];
    int32_t cl[NPT], zz[NPT];
    uint32_t rmk[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int32_t j = k * PG_BS + tid;
      fit[k] = false; sc[k] = 0; raw[k] = 0; cnt[k] = 0; cl[k] = 0; zz[k] = -1; rmk[k] = 0;
      if (j >= nrows) continue;
      const int64_t i = lo + j;
      KsimRow r;
      r.ac = L.ac[j]; r.am = L.am[j]; r.rc = L.rc[j]; r.rm = L.rm[j]; r.zc = L.zc[j]; r.zm = L.zm[j];
      r.allowed = L.al[j]; r.count = L.ct[j]; r.fl = L.fl[j];
      const uint32_t st = g.d.n_st ? (uint32_t)L.st[(int64_t)P.cls * chunk + j] : pg_static_word(c, P.cls, L.ls[j], L.ts[j]);
      if (k == 0) PG_STAMP(8);
      const uint32_t m = pg_predicates<false>(c, g, L, X, P, H, j, i, r, st, PgHyp{});
      if (k == 0) PG_STAMP(9);
      rmk[k] = m;
      if (m) continue;
      fit[k] = true;
      sc[k] = ksim_map_score(c, P, r);
      if (k == 0) PG_STAMP(10);
      cl[k] = (k1 > 1 ? (int32_t)((st >> 4) & 15u) : 0) * k2 + (k2 > 1 ? (int32_t)((st >> 8) & 15u) : 0);
      if (ipa) raw[k] = pg_interpod_raw<false>(L, X, H, j, PgHyp{});
      if (sp >= 0) {
        cnt[k] = L.cnt[(int64_t)sp * chunk + j];
        zz[k] = g.A.zone_key >= 0 ? L.dom[(int64_t)g.A.zone_key * chunk + j] : -1;
      }
    }
    PG_STAMP(0);

    // ---- 2. pass A over the grid (pods that read InterPodAffinity / SelectorSpread / the
    //         auxiliary priority) ----
    if (ipa || sp >= 0 || ap >= 0) {
      int64_t mn = 0, mx = 0, smx = 0, hz = 0, amx = 0, atot = 0, ahz = 0;
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        if (!fit[k]) continue;
        mn = raw[k] < mn ? raw[k] : mn;
        mx = raw[k] > mx ? raw[k] : mx;
        smx = cnt[k] > smx ? cnt[k] : smx;
        if (zz[k] >= 0) {
          hz = 1;
          if (cnt[k]) atomicAdd(&s_z[zz[k]], (unsigned long long)cnt[k]);
        }
        if (ap >= 0) {  // the auxiliary priority (passa_reduce's): max, sum, haveZones, domain sums
          const int32_t j = k * PG_BS + tid;
          const int64_t v = L.cnt[(int64_t)ap * chunk + j];
          const int32_t d = L.dom[(int64_t)g.A.aux_key * chunk + j];
          amx = v > amx ? v : amx;
          atot += v;
          if (d >= 0) {
            ahz = 1;
            if (v) atomicAdd(&s_az[d], (unsigned long long)v);
          }
        }
      }
      if (ipa) { mn = ksimw::min_i64(mn); mx = ksimw::max_i64(mx); }
      if (sp >= 0) { smx = ksimw::max_i32((int32_t)smx); hz = __ballot(hz != 0) ? 1 : 0; }
      if (ap >= 0) { amx = ksimw::max_i64(amx); atot = ksimw::sum_i64(atot); ahz = __ballot(ahz != 0) ? 1 : 0; }
      if (lane == 0) {
        s_a[0][wv] = mn; s_a[1][wv] = mx; s_a[2][wv] = smx; s_a[3][wv] = hz;
        s_a[4][wv] = amx; s_a[5][wv] = atot; s_a[6][wv] = ahz;
      }
      __syncthreads();
      PG_STAMP(6);
      if (wv == 0) {
        const int nz = sp >= 0 ? g.n_zone : 0;
        const int na = ap >= 0 ? g.A.n_adom : 0;  // <= PG_MAXAD (host-checked)
        const int A0 = 4 + nz;                     // the auxiliary words
        const int RA = A0 + (ap >= 0 ? 3 + na : 0);
        // word w's combine: 0 = min, 1 = max, 2 = sum
        auto wop = [&](int w) { return w == 0 ? 0 : (w < 4 ? 1 : (w < A0 ? 2 : (w == A0 || w == A0 + 2 ? 1 : 2))); };
        // publish this workgroup's record (lane w = word w), tagged; the zone / domain sums are
        // reset for the next pod by the same lane that read them
        if (lane < RA) {
          int64_t v;
          if (lane < 4 || (lane >= A0 && lane < A0 + 3)) {
            const int row = lane < 4 ? lane : 4 + lane - A0;
            const int op = wop(lane);
            v = s_a[row][0];
#pragma unroll
            for (int w = 1; w < PG_NW; ++w) {
              const int64_t x = s_a[row][w];
              v = op == 0 ? (x < v ? x : v) : (op == 1 ? (x > v ? x : v) : v + x);
            }
          } else if (lane < A0) {
            v = (int64_t)s_z[lane - 4];
            s_z[lane - 4] = 0;
          } else {
            v = (int64_t)s_az[lane - A0 - 3];
            s_az[lane - A0 - 3] = 0;
          }
          pg_store(rec_at(g.gran, slot, lane, blockIdx.x), ((uint64_t)tag << 56) | ((uint64_t)(v + B55) & M56));
        }
        // sweep every record: lane l reads workgroups l, l + 64, ...; batches of 8 words
        int64_t a_mn = 0, a_mx = 0, a_smx = 0, a_hz = 0, a_amx = 0, a_atot = 0, a_ahz = 0;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool ok = true;
        for (int w0 = 0; w0 < RA && ok; w0 += 8) {
          uint64_t v[8][MB];
          for (;;) {
            bool mine = true;
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
              for (int m = 0; m < MB; ++m) {
                const int b = lane + 64 * m;
                v[u][m] = (w0 + u < RA && b < G) ? pg_load(rec_at(g.gran, slot, w0 + u, b)) : ((uint64_t)tag << 56);
                mine &= gtag(v[u][m]) == tag;
              }
            if (__all(mine)) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > g.spin_ticks) { ok = false; break; }
            __builtin_amdgcn_s_sleep(1);
          }
          if (!ok) break;
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int word = w0 + u;
            if (word >= RA) break;
            const int op = wop(word);
            int64_t acc = op == 0 ? INT64_MAX : (op == 1 ? INT64_MIN : 0);
#pragma unroll
            for (int m = 0; m < MB; ++m) {
              if (lane + 64 * m >= G) continue;
              const int64_t x = (int64_t)(v[u][m] & M56) - B55;
              if (op == 0) acc = x < acc ? x : acc;
              else if (op == 1) acc = x > acc ? x : acc;
              else acc += x;
            }
            if (word == 0) a_mn = ipa ? ksimw::min_i64(acc) : 0;
            else if (word == 1) a_mx = ipa ? ksimw::max_i64(acc) : 0;
            else if (word == 2) a_smx = sp >= 0 ? ksimw::max_i64(acc) : 0;
            else if (word == 3) a_hz = sp >= 0 ? ksimw::max_i64(acc) : 0;
            else if (word < A0) {
              const int64_t zsum = ksimw::sum_i64(acc);
              if (lane == 0) s_gz[word - 4] = zsum;
            } else if (word == A0) a_amx = ksimw::max_i64(acc);
            else if (word == A0 + 1) a_atot = ksimw::sum_i64(acc);
            else if (word == A0 + 2) a_ahz = ksimw::max_i64(acc);
            else {
              const int64_t dsum = ksimw::sum_i64(acc);
              if (lane == 0) s_gaz[word - A0 - 3] = dsum;
            }
          }
        }
        if (!ok) {
          if (lane == 0) { atomicOr(c.err, 4); s_abort = 1; }
        } else if (lane == 0) {
          s_g[0] = a_mn < 0 ? a_mn : 0;  // the accumulators start at 0 (interpod_affinity.go:129-131)
          s_g[1] = a_mx > 0 ? a_mx : 0;
          s_g[2] = a_smx; s_g[3] = a_hz;
          int64_t zm = 0;
          for (int z = 0; z < nz; ++z) zm = s_gz[z] > zm ? s_gz[z] : zm;
          s_g[4] = zm;
          int64_t am = 0;  // (over every domain: zeros included, as passa_reduce)
          for (int z = 0; z < na; ++z) am = s_gaz[z] > am ? s_gaz[z] : am;
          s_g[5] = a_amx; s_g[6] = a_atot; s_g[7] = a_ahz; s_g[8] = am;
        }
      }
      __syncthreads();
      if (s_abort) { stop_pod = pod; break; }
      const int64_t gmn = s_g[0], gmx = s_g[1], gsmx = s_g[2], ghz = s_g[3], gzm = s_g[4];
      const int64_t gamx = s_g[5], gatot = s_g[6], gahz = s_g[7], gazm = s_g[8];
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        if (!fit[k]) continue;
        if (ipa)
          sc[k] = (int64_t)((uint64_t)sc[k] +
                            (uint64_t)c.w[KSIM_W_INTERPOD_AFFINITY] * (uint64_t)ksim_interpod_score(raw[k], gmn, gmx));
        if (sp >= 0)
          sc[k] = (int64_t)((uint64_t)sc[k] + (uint64_t)c.w[KSIM_W_SELECTOR_SPREAD] *
                                                  (uint64_t)ksim_spread_score(cnt[k], gsmx, ghz != 0, zz[k],
                                                                              zz[k] >= 0 ? s_gz[zz[k]] : 0, gzm));
        if (ap >= 0) {  // (aux_add's; count and domain from the rows' LDS image)
          const int32_t j = k * PG_BS + tid;
          const int32_t d = L.dom[(int64_t)g.A.aux_key * chunk + j];
          const int64_t v = L.cnt[(int64_t)ap * chunk + j];
          const int64_t ds = d >= 0 ? s_gaz[d] : 0;
          sc[k] = (int64_t)((uint64_t)sc[k] + (uint64_t)g.A.aux_w * (uint64_t)ksim_aux_score(g.A.aux_kind, v, d, ds, gamx, gatot,
                                                                                           gahz != 0, gazm));
        }
      }
    }
    if (aon && ap < 0) {  // serviceAntiAffinity of a pod no service selects: 10 on a labelled row (no pass A)
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        if (!fit[k]) continue;
        const int32_t d = L.dom[(int64_t)g.A.aux_key * chunk + k * PG_BS + tid];
        sc[k] = (int64_t)((uint64_t)sc[k] + (uint64_t)g.A.aux_w * (uint64_t)ksim_aux_score(g.A.aux_kind, 0, d, 0, 0, 0, false, 0));
      }
    }
    PG_STAMP(1);

    // ---- 3. per reduce class (max, count) and fit count of this workgroup ----
    int32_t nf = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) nf += __popcll(__ballot(fit[k]));
    if (lane == 0) s_fit[wv] = nf;
    for (int q = 0; q < K; ++q) {
      int32_t v = -1;
#pragma unroll
      for (int k = 0; k < NPT; ++k)
        if (fit[k] && cl[k] == q && (int32_t)sc[k] > v) v = (int32_t)sc[k];
      const int32_t wm = ksimw::max_i32(v);
      int32_t cn = 0;
#pragma unroll
      for (int k = 0; k < NPT; ++k) cn += __popcll(__ballot(fit[k] && cl[k] == q && (int32_t)sc[k] == wm));
      if (lane == 0) { s_mx[wv][q] = wm; s_cn[wv][q] = wm < 0 ? 0 : cn; }
    }
    __syncthreads();
    PG_STAMP(2);

    // ---- 4. wave 0: publish, sweep every workgroup's granules, decide; waves 1-3: prefetch ----
    if (wv == 0) {
      if (lane < K) {
        int32_t m = -1, nn = 0, f = 0;
#pragma unroll
        for (int w = 0; w < PG_NW; ++w) {
          f += s_fit[w];
          if (!s_cn[w][lane]) continue;
          if (s_mx[w][lane] > m) { m = s_mx[w][lane]; nn = s_cn[w][lane]; }
          else if (s_mx[w][lane] == m) nn += s_cn[w][lane];
        }
        const uint64_t v = ((uint64_t)tag << 56) | (lane == 0 ? ((uint64_t)f << 44) : 0) | ((uint64_t)nn << 32) |
                           (uint64_t)(uint32_t)m;
        pg_store(cls_at(g.gran, slot, lane, blockIdx.x), v);
      }
      // the decision's per-class map values (lane q = reduce class q)
      int64_t tv_l = 0, av_l = 0, ad_l = 0;
      if (lane < K) {
        tv_l = X.tv(K > 1 ? lane / k2 : 0);
        av_l = X.av(K > 1 ? lane % k2 : 0);
        ad_l = X.ad(K > 1 ? lane % k2 : 0);
      }
      int mode = 0, blk = -1, rank = 0;
      uint32_t win = 0;
      int32_t tgt_l = -2;  // lane q: class q's maximum if q wins
      // the workgroup holding the ix-th match from the top (lane-major workgroup order: lane l
      // holds l, l + 64, ...; name rank grows with the workgroup index), bm = matches per workgroup
      auto locate = [&](const int32_t (&bm)[MB], int64_t ix) {
        // matches in workgroups above b = (lanes above, same m) + (every lane, higher m)
        int64_t above = 0;
        int found = -1, rk = 0;
#pragma unroll
        for (int m = MB - 1; m >= 0; --m) {
        if (found < 0 && 64 * m < G) {
          const int32_t pre = ksimw::prefix_incl_i32(bm[m]);
          const int32_t tot = __builtin_amdgcn_readlane(pre, 63);
          const int64_t ab = above + (int64_t)(tot - pre);
          const bool hit = bm[m] > 0 && ix >= ab && ix < ab + bm[m];
          const uint64_t hb = __ballot(hit);
          if (hb) {
            const int src = __builtin_ffsll((long long)hb) - 1;
            found = src + 64 * m;
            rk = (int)__builtin_amdgcn_readlane((int32_t)(ix - ab), src);
          }
          above += tot;
        }
        }
        if (found < 0) { mode = -1; if (lane == 0) atomicOr(c.err, 2); }
        blk = found;
        rank = rk;
      };
      if (K == 1) {
        // one reduce class (no TaintToleration / NodeAffinity spread among the fit nodes): the
        // class maximum is the best total, and only granule 0 of each workgroup is read
        uint64_t gv0[MB];
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool ok = false;
        for (;;) {
          bool mine = true;
#pragma unroll
          for (int m = 0; m < MB; ++m) {
            const int b = lane + 64 * m;
            gv0[m] = b < G ? pg_load(cls_at(g.gran, slot, 0, b)) : ((uint64_t)tag << 56);
            mine &= gtag(gv0[m]) == tag;
          }
          if (__all(mine)) { ok = true; break; }
          if (__builtin_amdgcn_s_memrealtime() - t0 > g.spin_ticks) break;
          __builtin_amdgcn_s_sleep(1);
        }
#ifdef KSIM_STAMPS
        if (blockIdx.x == 0 && tid == 0) PG_STAMP(7);
#endif
        if (!ok) {
          mode = -1;
          if (lane == 0) atomicOr(c.err, 4);
        } else {
          int32_t f = 0, mm = -1, cc = 0;
#pragma unroll
          for (int m = 0; m < MB; ++m) {
            if (lane + 64 * m >= G) continue;
            f += gfit(gv0[m]);
            const int32_t cn = gcnt(gv0[m]), sc0 = gscore(gv0[m]);
            if (!cn) continue;
            if (sc0 > mm) { mm = sc0; cc = cn; }
            else if (sc0 == mm) cc += cn;
          }
          const int32_t F = ksimw::sum_i32(f);
          if (F > 0) {
            mode = 1;
            int64_t ix = 0;
            int32_t M0 = -1;
            if (F > 1) {  // generic_scheduler.go:153-156: a single fit skips selectHost
              mode = 2;
              M0 = ksimw::max_i32(cc ? mm : -1);
              const int32_t C = ksimw::sum_i32((cc && mm == M0) ? cc : 0);
              win = 1;
              tgt_l = lane == 0 ? M0 : -2;
              ix = (counter >> 32) ? (int64_t)(counter % (uint64_t)C) : (int64_t)((uint32_t)counter % (uint32_t)C);
              counter += 1;  // generic_scheduler.go:192-195
            }
            int32_t bm[MB];
#pragma unroll
            for (int m = 0; m < MB; ++m) {
              int32_t sb = 0;
              if (lane + 64 * m < G)
                sb = mode == 1 ? gfit(gv0[m]) : ((gcnt(gv0[m]) && gscore(gv0[m]) == M0) ? gcnt(gv0[m]) : 0);
              bm[m] = sb;
            }
            locate(bm, ix);
          }
        }
      } else {
        uint64_t gv[KSIM_MAX_RCLASS][MB];
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool ok = false;
        for (;;) {
          bool mine = true;
#pragma unroll
          for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
#pragma unroll
            for (int m = 0; m < MB; ++m) {
              const int b = lane + 64 * m;
              gv[q][m] = (q < K && b < G) ? pg_load(cls_at(g.gran, slot, q, b)) : ((uint64_t)tag << 56);
              mine &= gtag(gv[q][m]) == tag;
            }
          }
          if (__all(mine)) { ok = true; break; }
          if (__builtin_amdgcn_s_memrealtime() - t0 > g.spin_ticks) break;
          __builtin_amdgcn_s_sleep(1);
        }
#ifdef KSIM_STAMPS
        if (blockIdx.x == 0 && tid == 0) PG_STAMP(7);
#endif
        if (!ok) {
          mode = -1;
          if (lane == 0) atomicOr(c.err, 4);
        } else {
          int32_t F = 0;
          int32_t mq_l = -1, cq_l = 0;  // lane q: class q's global maximum and its count
          int32_t f = 0;
#pragma unroll
          for (int m = 0; m < MB; ++m) f += (lane + 64 * m < G) ? gfit(gv[0][m]) : 0;
          F = ksimw::sum_i32(f);
#pragma unroll
          for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
            if (q < K) {
              int32_t mm = -1, cc = 0;
#pragma unroll
              for (int m = 0; m < MB; ++m) {
                if (lane + 64 * m >= G) continue;
                const int32_t cn = gcnt(gv[q][m]), s = gscore(gv[q][m]);
                if (!cn) continue;
                if (s > mm) { mm = s; cc = cn; }
                else if (s == mm) cc += cn;
              }
              const int32_t Mq = ksimw::max_i32(cc ? mm : -1);
              const int32_t Cq = ksimw::sum_i32((cc && mm == Mq) ? cc : 0);
              mq_l = lane == q ? Mq : mq_l;
              cq_l = lane == q ? Cq : cq_l;
            }
          }
#ifdef KSIM_STAMPS
          if (blockIdx.x == 0 && tid == 0) PG_STAMP(11);
#endif
          if (F > 0) {
            mode = 1;
            int64_t ix = 0;
            if (F > 1) {  // generic_scheduler.go:153-156: a single fit skips selectHost
              mode = 2;
              // lane q = reduce class q: NormalizeReduce over the filtered set, weighted totals
              // (reduce.go:29-64, generic_scheduler.go:632-639), the best total and its classes
              const bool live = lane < K && cq_l != 0;
              int64_t mxT = 0, mxA = 0;
              // K <= 16: the class lanes are one DPP row
              if (k1 > 1 || c.w[KSIM_W_TAINT_TOLERATION]) mxT = ksimw::max16_i64(live ? tv_l : 0);
              if (k2 > 1 || c.w[KSIM_W_NODE_AFFINITY]) mxA = ksimw::max16_i64(live ? av_l : 0);
              uint64_t t = (uint64_t)(int64_t)mq_l + (uint64_t)ad_l;
              if (c.w[KSIM_W_TAINT_TOLERATION]) t += (uint64_t)c.w[KSIM_W_TAINT_TOLERATION] * (uint64_t)ksim_norm(tv_l, mxT, true);
              if (c.w[KSIM_W_NODE_AFFINITY]) t += (uint64_t)c.w[KSIM_W_NODE_AFFINITY] * (uint64_t)ksim_norm(av_l, mxA, false);
              const int64_t tot = live ? (int64_t)t : INT64_MIN;
              const int64_t best = ksimw::max16_i64(tot);
              const uint64_t wbm = __ballot(live && tot == best);
              win = (uint32_t)wbm;
              const int32_t C = ksimw::sum16_i32(((wbm >> lane) & 1ull) ? cq_l : 0);
              tgt_l = ((wbm >> lane) & 1ull) ? mq_l : -2;
              ix = (counter >> 32) ? (int64_t)(counter % (uint64_t)C) : (int64_t)((uint32_t)counter % (uint32_t)C);
              counter += 1;  // generic_scheduler.go:192-195
            }
            // locate the workgroup holding the ix-th match from the top (lane-major workgroup order:
            // lane l holds l, l + 64, ...; name rank grows with the workgroup index)
            int32_t bm[MB];
#pragma unroll
            for (int m = 0; m < MB; ++m) {
              const int b = lane + 64 * m;
              int32_t s = 0;
              if (b < G) {
                if (mode == 1) {
                  s = gfit(gv[0][m]);
                } else {
#pragma unroll
                  for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
                    if (q < K && ((win >> q) & 1u)) {
                      const int32_t Mq = __builtin_amdgcn_readlane(mq_l, q);
                      if (gcnt(gv[q][m]) && gscore(gv[q][m]) == Mq) s += gcnt(gv[q][m]);
                    }
                  }
                }
              }
              bm[m] = s;
            }
            locate(bm, ix);
          }
        }
      }
#ifdef KSIM_STAMPS
      if (blockIdx.x == 0 && tid == 0) PG_STAMP(12);
#endif
      if (lane < KSIM_MAX_RCLASS) s_tgt[lane] = tgt_l;
      if (lane == 0) { s_mode = mode; s_blk = blk; s_rank = rank; s_win = win; s_node = -1; }
    } else if (pf) {
      uint4* dst = reinterpret_cast<uint4*>(xrec(pod + 1));
      const int t = tid - 64;
      if (t < pfw) dst[t] = pf0;
      if (t + 3 * 64 < pfw) dst[t + 3 * 64] = pf1;
    }
    __syncthreads();
    PG_STAMP(3);
    const int mode = s_mode;
    if (mode < 0) { stop_pod = pod; break; }  // uniform: every workgroup reached the same verdict

    // ---- 5. FitError: every workgroup adds its rows' reasons ----
    if (mode == 0) {
      if (c.collect && c.out_reasons) {
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          if (!__ballot(rmk[k] != 0)) continue;
          for (int r = 0; r < KSIM_NREASONS; ++r) {
            const int32_t nr = __popcll(__ballot((rmk[k] >> r) & 1u));
            if (lane == 0 && nr) atomicAdd(&c.out_reasons[pod * KSIM_NREASONS + r], nr);
          }
        }
      }
      if (blockIdx.x == 0 && tid == 0) c.out_node[pod] = -1;
      continue;  // nothing committed: the next pod reads the same state
    }

    // ---- 6. the owner picks the row (the rank-th match from the top, selectHost's order) from its
    //         threads' own evaluations, and the thread holding that row commits it ----
    const bool owner = s_blk == (int)blockIdx.x;
    const bool shared = (H.fl & PGF_SHARED) != 0;
    const bool aff_commit = (H.fl & PGF_AFF) && !c.no_commit;
    int ksel = -1;  // which of this thread's rows was chosen
    if (owner) {
      const uint32_t win = s_win;
      const int32_t rr = s_rank;
      bool mt[NPT];
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        mt[k] = fit[k] && (mode == 1 || (((win >> cl[k]) & 1u) && (int32_t)sc[k] == s_tgt[cl[k]]));
        const uint64_t bl = __ballot(mt[k]);
        if (lane == 0) s_bal[k][wv] = bl;
      }
      __syncthreads();
      // matches above row k*256 + wv*64 + lane: every wave's in higher k, higher waves' in this
      // k, higher lanes' in this wave
      int32_t above = 0;
#pragma unroll
      for (int k = NPT - 1; k >= 0; --k) {
        int32_t up = 0;
#pragma unroll
        for (int w = PG_NW - 1; w >= 0; --w)
          if (w > wv) up += __popcll(s_bal[k][w]);
        const int32_t mine = __popcll((s_bal[k][wv] >> lane) >> 1);
        if (mt[k] && above + up + mine == rr) ksel = k;
#pragma unroll
        for (int w = 0; w < PG_NW; ++w) above += __popcll(s_bal[k][w]);
      }
      if (rr >= above) {  // every thread of the owner computed the same total: a uniform exit
        if (tid == 0) atomicOr(c.err, 2);
        break;
      }
    }
    if (ksel >= 0) {
      const int32_t jsel = ksel * PG_BS + tid;
      const int64_t w = lo + jsel;
      const ksim_pod& Pr = X.pod();
      c.out_node[pod] = (int32_t)w;
      if (shared) {
        s_node = w;
        if (g.svc_on && aff_commit && Pr.aff_ident > 0) {
          // the lenders' disagreements before the counts move, released ahead of the commit word
          // the other workgroups acquire before their next evaluation reads them
          pg_svc_commit(g, L, Pr.aff_ident, jsel);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        }
        pg_store(g.gran + PG_COMMIT_OFF + slot, ((uint64_t)tag << 56) | (uint64_t)w);
      }
      if (!c.no_commit) {
        // NodeInfo.AddPod on the row (node_info.go:318-341)
        L.rc[jsel] += Pr.add_cpu; L.rm[jsel] += Pr.add_mem; L.zc[jsel] += P.nz_cpu; L.zm[jsel] += P.nz_mem;
        L.ct[jsel] += 1;
        const int64_t agpu = Pr.add_gpu, aeph = Pr.add_eph;
        if (agpu | aeph) {
          const int64_t gg = c.req_gpu[w] + agpu, ge = c.req_eph[w] + aeph;
          c.req_gpu[w] = gg;
          c.req_eph[w] = ge;
          uint32_t fl = L.fl[jsel] & ~(KSIM_N_GPU_OVER | KSIM_N_EPH_OVER);
          if (c.alloc_gpu[w] < gg) fl |= KSIM_N_GPU_OVER;
          if (c.alloc_eph[w] < ge) fl |= KSIM_N_EPH_OVER;
          L.fl[jsel] = fl;
        }
        const ksim_scalar_req* sr = X.sec<ksim_scalar_req>(PGS_SCAL);
        for (int32_t s = 0; s < H.n_scal; ++s) c.req_scalar[(int64_t)sr[s].col * n + w] += sr[s].add;
        // HostPortInfo.Add (utils.go:45-60)
        const uint64_t* pk = X.sec<uint64_t>(PGS_PORT);
        for (int32_t k = 0; k < H.n_port; ++k) {
          const uint64_t key = pk[k];
          const int32_t cnt0 = psl ? L.pc[jsel] : 0;
          bool dup = false;
          for (int32_t s = 0; s < cnt0; ++s)
            if (L.pk[(int64_t)s * chunk + jsel] == key) { dup = true; break; }
          if (dup) continue;
          if (cnt0 >= psl) { atomicOr(c.err, 1); continue; }
          L.pk[(int64_t)cnt0 * chunk + jsel] = key;
          L.pc[jsel] = cnt0 + 1;
        }
        // the pod's volume mounts (ksim_vol_commit with sign +1)
        if (H.fl & PGF_VOL) {
          const int4* refs = X.sec<int4>(PGS_REF);
          for (int32_t x = 0; x < H.n_ref; ++x) {
            const int4 ref = refs[x];
            const uint32_t f = (uint32_t)ref.y;
            const int sh = (f & KSIM_VOL_VIA_PVC) ? 22 : (f & KSIM_VOL_READ_ONLY) ? 11 : 0;
            const uint64_t fmask = (sh == 22 ? 0x3FFull : 0x7FFull) << sh;
            const uint64_t one = 1ull << sh;
            const int32_t cnt0 = vcap ? L.vc[jsel] : 0;
            const int32_t s = pg_vol_find(g, L, jsel, w, cnt0, ref.x);
            if (s >= 0) {
              uint64_t& sw = *pg_slot(g, L, jsel, w, s);
              if ((sw & fmask) == fmask) atomicOr(c.err, 1);
              else sw += one;
            } else if (cnt0 >= vcap) {
              atomicOr(c.err, 1);
            } else {
              *pg_slot(g, L, jsel, w, cnt0) = ((uint64_t)(uint32_t)ref.x << 32) | one;
              L.vc[jsel] = cnt0 + 1;
              const uint32_t kf = (uint32_t)ref.z;
#pragma unroll
              for (int t = 0; t < 3; ++t)
                if ((kf >> t) & 1u) L.vh[(int64_t)t * chunk + jsel] += 1;
            }
          }
        }
        if (aff_commit && !shared) {
          // the pod's counts on node-like keys: only its own row changes
          const int2* mp = X.sec<int2>(PGS_MP);
          for (int32_t x = 0; x < H.n_mp; ++x)
            if (L.dom[(int64_t)mp[x].y * chunk + jsel] >= 0) L.cnt[(int64_t)mp[x].x * chunk + jsel] += 1;
          const PgCar* cr = X.sec<PgCar>(PGS_CAR);
          for (int32_t x = 0; x < H.n_car; ++x)
            if (L.dom[(int64_t)cr[x].key * chunk + jsel] >= 0) L.car[(int64_t)cr[x].term * chunk + jsel] += cr[x].amount;
        }
      }
    }
    PG_STAMP(4);
    // ---- 7. shared topology domains: every workgroup applies the pod's counts to its rows of
    //         the chosen node's domains (NodeInfo.AddPod's affinity part, replicated) ----
    if (shared && aff_commit) {
      if (!owner && tid == 0) {
        // the chosen node, from the owner's commit word
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint64_t v;
        while (gtag(v = pg_load(g.gran + PG_COMMIT_OFF + slot)) != tag) {
          if (__builtin_amdgcn_s_memrealtime() - t0 > g.spin_ticks) { atomicOr(c.err, 4); s_abort = 1; break; }
          __builtin_amdgcn_s_sleep(1);
        }
        if (g.svc_on) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (the owner's svc_conflict bits)
        s_node = (int64_t)(v & M56);
      }
      __syncthreads();
      if (s_abort) { stop_pod = pod; break; }
      const int64_t w = s_node;
      const int2* mp = X.sec<int2>(PGS_MP);
      const PgCar* cr = X.sec<PgCar>(PGS_CAR);
      const int32_t nm = H.n_mp, ncr = H.n_car;
      for (int32_t x = tid; x < nm + ncr; x += PG_BS) {
        const int32_t key = x < nm ? mp[x].y : cr[x - nm].key;
        s_dw[x] = g.A.dom[(int64_t)key * n + w];
      }
      __syncthreads();
      if (g.svc_on)  // the domain-0 copies: the pod's pairs on keys where the node is in domain 0
        for (int32_t x = tid; x < nm; x += PG_BS)
          if (s_dw[x] == 0) atomicAdd(&s_g0[mp[x].x], 1);
      for (int32_t y = tid; y < (nm + ncr) * nrows; y += PG_BS) {
        const int32_t x = y / nrows, j = y - x * nrows;
        const int32_t dw = s_dw[x];
        if (dw < 0) continue;
        if (x < nm) {
          if (L.dom[(int64_t)mp[x].y * chunk + j] == dw) L.cnt[(int64_t)mp[x].x * chunk + j] += 1;
        } else {
          const PgCar& k = cr[x - nm];
          if (L.dom[(int64_t)k.key * chunk + j] == dw)
            atomicAdd(reinterpret_cast<unsigned long long*>(&L.car[(int64_t)k.term * chunk + j]), (unsigned long long)k.amount);
        }
      }
      __syncthreads();
    }
    PG_STAMP(5);
  }
  // ---- the table is authoritative in HBM between calls: write the owned rows back ----
  pg_write_back(c, g, L, lo, nrows, chunk, tid, blockDim.x);
  if (tid == 0 && stop_pod < c.end) atomicMin((unsigned long long*)c.cursor, (unsigned long long)stop_pod);
  if (blockIdx.x == 0 && tid == 0) {
    *c.counter = counter;
    (void)0;  // the cursor: c.end preset by the host, lowered below by an aborting workgroup
#ifdef KSIM_STAMPS
    for (int k = 0; k < 16; ++k) c.dbg[k] += st_acc[k];
#endif
  }
}

// ===================================================================================================
// The dual-hypothesis form (the default): wave 0 is the control wave (exchange, decision), waves 1-3
// own the rows (row j = k * 192 + thread - 64).  While wave 0 sweeps pod p's class granules and
// decides, the row threads evaluate pod p+1 on every row twice — as the row stands (E0) and with
// pod p committed to it (E1, PgHyp) — so after the decision the owner's selected row swaps in its E1
// entry and every other row keeps E0: no evaluation sits between one decision and the next pass-A
// reduction.  The commit itself is deferred into the next exchange window.  Pods whose commit
// leaves the row's LDS image (gpu / ephemeral / scalar requests, shared-domain affinity counts) are
// no hypotheses (PGF_NOHYP): their node is committed at once and pod p+1 re-evaluated.
#define PG2_BS 512
#define PG2_NW (PG2_BS / 64)
#define PG_RT 192  // rows per thread slot: waves 1-3 (E0, the row state), waves 5-7 (E1)
#define PG_RW 3

struct PgEv {
  int64_t sc, raw;
  int32_t cnt, cl, zz;
  uint32_t rmk;
  bool fit;
  int32_t acnt;  // the auxiliary priority's count (PGF_AUX with a pair)
};
static_assert(sizeof(PgEv) == PG_EV_BYTES, "PgEv layout");

namespace {

template <bool HYP, bool AUX = false>
__device__ __forceinline__ PgEv pg_eval(const KsimCtx& c, const PGenArgs& g, const PgL& L, const PgX& X, const ksim_pod& P,
                                        const PgHdr& H, int32_t j, int64_t i, const PgHyp& y, const ksim_pod& Py,
                                        uint64_t* sa = nullptr) {
  PgEv e{0, 0, 0, 0, -1, 0, false};
#ifdef KSIM_STAMPS
  uint64_t t0_ = __builtin_amdgcn_s_memtime();
#endif
  KsimRow r;
  r.ac = L.ac[j]; r.am = L.am[j]; r.rc = L.rc[j]; r.rm = L.rm[j]; r.zc = L.zc[j]; r.zm = L.zm[j];
  r.allowed = L.al[j]; r.count = L.ct[j]; r.fl = L.fl[j];
  if (HYP) {  // NodeInfo.AddPod of the hypothesis (node_info.go:318-341): requests, non-zero requests, count
    const ksim_pod& Pr = y.X->pod();  // add_* are not in the uniform copy
    r.rc += Pr.add_cpu; r.rm += Pr.add_mem; r.zc += Py.nz_cpu; r.zm += Py.nz_mem; r.count += 1;
  }
  const uint32_t st = g.d.n_st ? (uint32_t)L.st[(int64_t)P.cls * L.chunk + j] : pg_static_word(c, P.cls, L.ls[j], L.ts[j]);
#ifdef KSIM_STAMPS
  if (sa) sa[0] += __builtin_amdgcn_s_memtime() - t0_;
#endif
  const uint32_t m = pg_predicates<HYP>(c, g, L, X, P, H, j, i, r, st, y, sa);
#ifdef KSIM_STAMPS
  t0_ = __builtin_amdgcn_s_memtime();
#endif
  e.rmk = m;
  if (m) return e;
  e.fit = true;
  e.sc = ksim_map_score(c, P, r);
  e.cl = (H.k1 > 1 ? (int32_t)((st >> 4) & 15u) : 0) * H.k2 + (H.k2 > 1 ? (int32_t)((st >> 8) & 15u) : 0);
  if (H.fl & PGF_IPA) e.raw = pg_interpod_raw<HYP>(L, X, H, j, y);
  if (H.sp >= 0) {
    e.cnt = pg_cnt<HYP>(L, y, H.sp, j);
    e.zz = g.A.zone_key >= 0 ? L.dom[(int64_t)g.A.zone_key * L.chunk + j] : -1;
  }
  if (AUX && (H.fl & PGF_AUX)) {
    const int32_t ap = (H.fl >> PGF_AUX_SHIFT) - 1;
    if (ap >= 0) e.acnt = pg_cnt<HYP>(L, y, ap, j);
  }
#ifdef KSIM_STAMPS
  if (sa) sa[5] += __builtin_amdgcn_s_memtime() - t0_;
#endif
  return e;
}

// NodeInfo.AddPod of pod (X, P, H) on row jsel = node w, on the LDS image (+ HBM side columns):
// resources, gpu / ephemeral / scalar requests, host ports, volume mounts and — unless the counts
// live in shared domains (applied by every workgroup) — the pod's affinity counts on its row.
__device__ __forceinline__ void pg_commit_row(const KsimCtx& c, const PGenArgs& g, const PgL& L, const PgX& X,
                                              const PgHdr& H, int32_t jsel, int64_t w) {
  const ksim_pod& Pr = X.pod();
  const int64_t n = c.n, chunk = L.chunk;
  L.rc[jsel] += Pr.add_cpu; L.rm[jsel] += Pr.add_mem; L.zc[jsel] += Pr.nz_cpu; L.zm[jsel] += Pr.nz_mem;
  L.ct[jsel] += 1;
  const int64_t agpu = Pr.add_gpu, aeph = Pr.add_eph;
  if (agpu | aeph) {
    const int64_t gg = c.req_gpu[w] + agpu, ge = c.req_eph[w] + aeph;
    c.req_gpu[w] = gg;
    c.req_eph[w] = ge;
    uint32_t fl = L.fl[jsel] & ~(KSIM_N_GPU_OVER | KSIM_N_EPH_OVER);
    if (c.alloc_gpu[w] < gg) fl |= KSIM_N_GPU_OVER;
    if (c.alloc_eph[w] < ge) fl |= KSIM_N_EPH_OVER;
    L.fl[jsel] = fl;
  }
  const ksim_scalar_req* sr = X.sec<ksim_scalar_req>(PGS_SCAL);
  for (int32_t s = 0; s < H.n_scal; ++s) c.req_scalar[(int64_t)sr[s].col * n + w] += sr[s].add;
  // HostPortInfo.Add (utils.go:45-60)
  const int32_t psl = g.d.pslots, vcap = g.d.vcap;
  const uint64_t* pk = X.sec<uint64_t>(PGS_PORT);
  for (int32_t k = 0; k < H.n_port; ++k) {
    const uint64_t key = pk[k];
    const int32_t cnt0 = psl ? L.pc[jsel] : 0;
    bool dup = false;
    for (int32_t s = 0; s < cnt0; ++s)
      if (L.pk[(int64_t)s * chunk + jsel] == key) { dup = true; break; }
    if (dup) continue;
    if (cnt0 >= psl) { atomicOr(c.err, 1); continue; }
    L.pk[(int64_t)cnt0 * chunk + jsel] = key;
    L.pc[jsel] = cnt0 + 1;
  }
  if (H.fl & PGF_VOL) {  // ksim_vol_commit with sign +1
    const int4* refs = X.sec<int4>(PGS_REF);
    for (int32_t x = 0; x < H.n_ref; ++x) {
      const int4 ref = refs[x];
      const uint32_t f = (uint32_t)ref.y;
      const int sh = (f & KSIM_VOL_VIA_PVC) ? 22 : (f & KSIM_VOL_READ_ONLY) ? 11 : 0;
      const uint64_t fmask = (sh == 22 ? 0x3FFull : 0x7FFull) << sh;
      const uint64_t one = 1ull << sh;
      const int32_t cnt0 = vcap ? L.vc[jsel] : 0;
      const int32_t s = pg_vol_find(g, L, jsel, w, cnt0, ref.x);
      if (s >= 0) {
        uint64_t& sw = *pg_slot(g, L, jsel, w, s);
        if ((sw & fmask) == fmask) atomicOr(c.err, 1);
        else sw += one;
      } else if (cnt0 >= vcap) {
        atomicOr(c.err, 1);
      } else {
        *pg_slot(g, L, jsel, w, cnt0) = ((uint64_t)(uint32_t)ref.x << 32) | one;
        L.vc[jsel] = cnt0 + 1;
        const uint32_t kf = (uint32_t)ref.z;
        for (int t = 0; t < 3; ++t)
          if ((kf >> t) & 1u) L.vh[(int64_t)t * chunk + jsel] += 1;
      }
    }
  }
  if ((H.fl & PGF_AFF) && !(H.fl & PGF_SHARED)) {  // node-like keys: only this row's counts change
    const int2* mp = X.sec<int2>(PGS_MP);
    for (int32_t x = 0; x < H.n_mp; ++x)
      if (L.dom[(int64_t)mp[x].y * chunk + jsel] >= 0) L.cnt[(int64_t)mp[x].x * chunk + jsel] += 1;
    const PgCar* cr = X.sec<PgCar>(PGS_CAR);
    for (int32_t x = 0; x < H.n_car; ++x)
      if (L.dom[(int64_t)cr[x].key * chunk + jsel] >= 0) L.car[(int64_t)cr[x].term * chunk + jsel] += cr[x].amount;
  }
}

// Reduce within each group of 8 lanes (every lane of the group gets the group's result): op 0 min,
// 1 max, 2 sum, per lane.
__device__ __forceinline__ int64_t pg_red8_step(int64_t acc, int64_t t, int op) {
  return op == 0 ? (t < acc ? t : acc) : (op == 1 ? (t > acc ? t : acc) : acc + t);
}
__device__ __forceinline__ int64_t pg_red8(int64_t acc, int op) {
  acc = pg_red8_step(acc, ksimw::dpp64<ksimw::QP_1032>(acc, acc), op);
  acc = pg_red8_step(acc, ksimw::dpp64<ksimw::QP_2301>(acc, acc), op);
  acc = pg_red8_step(acc, ksimw::dpp64<ksimw::ROW_HALF_MIRROR>(acc, acc), op);
  return acc;
}

__device__ __forceinline__ char* pg_xrec4(char* sm, const PGenArgs& g, int64_t r) {
  return sm + g.off[PGO_X0] + (uint32_t)(r & 3) * (g.off[PGO_X1] - g.off[PGO_X0]);
}

}  // namespace

template <int NPT, int MB, bool AUX>
__global__ __launch_bounds__(PG2_BS) void ksim_pgen2_kernel(KsimCtx c_arg, PGenArgs g_arg) {
  extern __shared__ __attribute__((aligned(16))) char pg_smem[];
  __shared__ int64_t s_a[7][PG2_NW];                  // pass A per wave: min, max, max count, haveZones, aux max / sum / haveZones
  __shared__ unsigned long long s_z[PG_MAXZ];        // pass A zone sums of this workgroup
  __shared__ unsigned long long s_az[PG_MAXAD];      // the auxiliary priority's domain sums of this workgroup
  __shared__ int64_t s_g[9];                         // pass A over the grid (+ aux max, sum, haveZones, max domain sum)
  __shared__ int64_t s_gz[PG_MAXZ];                  // countsByZone over the grid
  __shared__ int64_t s_gaz[PG_MAXAD];                // the auxiliary domain sums over the grid
  __shared__ int32_t s_mx[PG2_NW][KSIM_MAX_RCLASS];  // class partials per wave (only waves 1-3 hold rows)
  __shared__ int32_t s_cn[PG2_NW][KSIM_MAX_RCLASS];
  __shared__ int32_t s_fit[PG2_NW];
  __shared__ int32_t s_mode, s_blk, s_rank, s_abort;
  __shared__ uint32_t s_win;
  __shared__ int32_t s_tgt[KSIM_MAX_RCLASS];
  __shared__ int64_t s_node;
  __shared__ int32_t s_dw[PG_MAXL * 2];
  __shared__ uint64_t s_bal[NPT][PG_RW];             // owner: each row wave's ballot of its rows at the chosen score
#ifdef KSIM_STAMPS
  uint64_t st_acc[16] = {};
  uint64_t t_prev = __builtin_amdgcn_s_memtime();
  uint64_t ev_acc = 0, ev_acc1 = 0;  // threads 64 / 320: their rows' E0 / E1 evaluations
  uint64_t ev_sa[6] = {};
  uint64_t cm_acc = 0, cm_n = 0, ps_acc = 0, pr_acc = 0, cs_acc = 0, t_pub = 0;
#endif
  const KsimCtx& c = c_arg;
  const PGenArgs& g = g_arg;
  if (g.test_stall && blockIdx.x == gridDim.x - 1) return;  // diagnostic: a workgroup that never ran
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const bool rowt = wv >= 1 && wv <= 3;  // E0: the row state
  const bool hypt = wv >= 5;             // E1: the same rows under the hypothesis
  const int rt = rowt ? tid - 64 : tid - 320;
  const int G = gridDim.x;
  const int64_t chunk = c.chunk;
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = (lo + chunk < c.n) ? lo + chunk : c.n;
  const int32_t nrows = (int32_t)(hi - lo);
  const int64_t n = c.n;
  const PgL L = pg_lds(pg_smem, g, chunk);
  auto xrec = [&](int64_t r) { return pg_xrec4(pg_smem, g, r); };
  PgEv* ev1 = reinterpret_cast<PgEv*>(pg_smem + g.off[PGO_E1]);

  pg_stage_rows(c, g, L, lo, nrows, chunk, tid, blockDim.x);
  for (int64_t q = c.first; q < c.end && q < c.first + 2; ++q) {  // the records of the first two pods
    const uint4* src = reinterpret_cast<const uint4*>(g.rec + (q - c.first) * (int64_t)g.d.rec_stride);
    uint4* dst = reinterpret_cast<uint4*>(xrec(q));
    for (int32_t x = tid; x < g.d.rec_stride / 16; x += PG2_BS) dst[x] = src[x];
  }
  if (tid == 0) s_abort = 0;
  if (tid < PG_MAXZ) s_z[tid] = 0;
  if (AUX && tid < PG_MAXAD) s_az[tid] = 0;
  uint64_t counter = *c.counter;  // replicated genericScheduler.lastNodeIndex (wave 0)
  __syncthreads();
  pg_stage_counts(c, g, L, nrows, chunk, tid, blockDim.x);
  if (L.hd) {
    for (int32_t x = tid; x < g.d.n_pair; x += PG2_BS) L.hd[x] = 0;
    for (int32_t x = tid; x < g.d.n_carry; x += PG2_BS) { L.hc[x] = 0; L.hk[x] = 0; }
  }
  __syncthreads();

  // pod `first` on every row, as the rows stand
  PgEv cur[NPT];
  {
    PgX X0;
    X0.base = xrec(c.first);
    const PgHdr H0 = pg_hdr_u(X0.hdr());
    pg_sections(H0, X0.so);
    const ksim_pod P0 = pg_pod_u(X0.pod());
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int32_t j = k * PG_RT + rt;
      cur[k] = PgEv{0, 0, 0, 0, -1, 0, false};
      if (rowt && j < nrows) cur[k] = pg_eval<false, AUX>(c, g, L, X0, P0, H0, j, lo + j, PgHyp{}, P0);
    }
  }
  int32_t pend_j = -1;   // deferred commit of pod pend_pod on row pend_j (its row thread)
  int64_t pend_pod = -1;

  int64_t stop_pod = c.end;  // first pod not scheduled (a spin bound ran out: the grid is not co-resident)
  for (int64_t pod = c.first; pod < c.end; ++pod) {
    PgX X;
    X.base = xrec(pod);
    const PgHdr H = pg_hdr_u(X.hdr());
    pg_sections(H, X.so);
    const ksim_pod P = pg_pod_u(X.pod());
    const int K = H.K, k1 = H.k1, k2 = H.k2;
    const bool ipa = (H.fl & PGF_IPA) != 0;
    const int32_t sp = H.sp;
    // AUX (an instantiation for handles with the auxiliary priority's tables): the pod may read it
    const bool aon = AUX && (H.fl & PGF_AUX) != 0;
    const int32_t ap = AUX ? (H.fl >> PGF_AUX_SHIFT) - 1 : -1;  // (-1 without PGF_AUX too)
    const uint32_t tag = (uint32_t)((pod - c.first + 1) & 0xFF);
    const int slot = (int)(pod % PG_NSLOT);
    const bool has_next = pod + 1 < c.end;
    // wave 4 copies pod p+2's record into LDS in the decision window (its buffer held pod p-2's)
    const bool pf = wv == 4 && pod + 2 < c.end;

    // ---- pass A over the grid (pods that read InterPodAffinity / SelectorSpread / the
    //      auxiliary priority with a pair) ----
    if (ipa || sp >= 0 || ap >= 0) {
      int64_t mn = 0, mx = 0, smx = 0, hz = 0, amx = 0, atot = 0, ahz = 0;
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        if (!cur[k].fit) continue;
        mn = cur[k].raw < mn ? cur[k].raw : mn;
        mx = cur[k].raw > mx ? cur[k].raw : mx;
        smx = cur[k].cnt > smx ? cur[k].cnt : smx;
        if (cur[k].zz >= 0) {
          hz = 1;
          if (cur[k].cnt) atomicAdd(&s_z[cur[k].zz], (unsigned long long)cur[k].cnt);
        }
        if (ap >= 0) {  // (passa_reduce's auxiliary words; the count as evaluated, E0 or E1)
          const int64_t v = cur[k].acnt;
          const int32_t d = L.dom[(int64_t)g.A.aux_key * chunk + k * PG_RT + rt];
          amx = v > amx ? v : amx;
          atot += v;
          if (d >= 0) {
            ahz = 1;
            if (v) atomicAdd(&s_az[d], (unsigned long long)v);
          }
        }
      }
      if (ipa) { mn = ksimw::min_i64(mn); mx = ksimw::max_i64(mx); }
      if (sp >= 0) { smx = ksimw::max_i32((int32_t)smx); hz = __ballot(hz != 0) ? 1 : 0; }
      if (ap >= 0) { amx = ksimw::max_i64(amx); atot = ksimw::sum_i64(atot); ahz = __ballot(ahz != 0) ? 1 : 0; }
      if (lane == 0) {
        s_a[0][wv] = mn; s_a[1][wv] = mx; s_a[2][wv] = smx; s_a[3][wv] = hz;
        if (AUX) { s_a[4][wv] = amx; s_a[5][wv] = atot; s_a[6][wv] = ahz; }
      }
      __syncthreads();
      PG_STAMP(6);
      if (wv == 0) {
        const int nz = sp >= 0 ? g.n_zone : 0;
        const int na = ap >= 0 ? g.A.n_adom : 0;  // <= PG_MAXAD (host-checked)
        const int A0 = 4 + nz;                     // the auxiliary words
        const int RA = A0 + (ap >= 0 ? 3 + na : 0);
        // word w's combine: 0 = min, 1 = max, 2 = sum
        auto wop = [&](int w) { return w == 0 ? 0 : (w < 4 ? 1 : ((!AUX || w < A0) ? 2 : (w == A0 || w == A0 + 2 ? 1 : 2))); };
        if (lane < RA) {
          int64_t v;
          if (lane < 4 || (AUX && lane >= A0 && lane < A0 + 3)) {
            const int row = lane < 4 ? lane : 4 + lane - A0;
            const int op = wop(lane);
            v = s_a[row][0];
#pragma unroll
            for (int w = 1; w < PG2_NW; ++w) {
              const int64_t x = s_a[row][w];
              v = op == 0 ? (x < v ? x : v) : (op == 1 ? (x > v ? x : v) : v + x);
            }
          } else if (!AUX || lane < A0) {
            v = (int64_t)s_z[lane - 4];
            s_z[lane - 4] = 0;
          } else {
            v = (int64_t)s_az[lane - A0 - 3];
            s_az[lane - A0 - 3] = 0;
          }
          pg_store(rec_at(g.gran, slot, lane, blockIdx.x), ((uint64_t)tag << 56) | ((uint64_t)(v + B55) & M56));
        }
#ifdef KSIM_STAMPS
        t_pub = __builtin_amdgcn_s_memtime();
#endif
        // transposed sweep: lane l reads word w0 + l / 8 of workgroups l % 8, l % 8 + 8, ... (G <= 64),
        // folds them, and one 3-step DPP chain within each group of 8 lanes reduces every word at once
        int64_t r0 = 0, zmax = 0, azmax = 0;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool ok = true;
        for (int w0 = 0; w0 < RA && ok; w0 += 8) {
          const int word = w0 + (lane >> 3);
          const bool wl = word < RA;
          uint64_t v[8];
          for (;;) {
            bool mine = true;
#pragma unroll
            for (int m = 0; m < 8; ++m) {
              const int b = (lane & 7) + 8 * m;
              v[m] = (wl && b < G) ? pg_load(rec_at(g.gran, slot, word, b)) : ((uint64_t)tag << 56);
              mine &= gtag(v[m]) == tag;
            }
            if (__all(mine)) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > g.spin_ticks) { ok = false; break; }
            __builtin_amdgcn_s_sleep(1);
          }
          if (!ok) break;
#ifdef KSIM_STAMPS
          {
            const uint64_t t_ = __builtin_amdgcn_s_memtime();
            ps_acc += t_ - t_pub;
            t_pub = t_;
          }
#endif
          const int op = wop(word);  // min, max, sum
          int64_t acc = op == 0 ? INT64_MAX : (op == 1 ? INT64_MIN : 0);
#pragma unroll
          for (int m = 0; m < 8; ++m) {
            if (!wl || (lane & 7) + 8 * m >= G) continue;
            const int64_t x = (int64_t)(v[m] & M56) - B55;
            acc = op == 0 ? (x < acc ? x : acc) : (op == 1 ? (x > acc ? x : acc) : acc + x);
          }
          acc = pg_red8(acc, op);
          if (w0 == 0) r0 = acc;
          if (wl && word >= 4 && (!AUX || word < A0)) {
            zmax = acc > zmax ? acc : zmax;
            if ((lane & 7) == 0) s_gz[word - 4] = acc;
          } else if (AUX && wl && word >= A0 && word < A0 + 3) {
            if ((lane & 7) == 0) s_g[5 + word - A0] = acc;
          } else if (AUX && wl && word >= A0 + 3) {
            azmax = acc > azmax ? acc : azmax;
            if ((lane & 7) == 0) s_gaz[word - A0 - 3] = acc;
          }
        }
        if (nz) zmax = ksimw::max_i64(zmax);
        if (na) azmax = ksimw::max_i64(azmax);
        const int64_t a_mn = ipa ? ksimw::readlane64(r0, 0) : 0, a_mx = ipa ? ksimw::readlane64(r0, 8) : 0;
        const int64_t a_smx = sp >= 0 ? ksimw::readlane64(r0, 16) : 0, a_hz = sp >= 0 ? ksimw::readlane64(r0, 24) : 0;
#ifdef KSIM_STAMPS
        pr_acc += __builtin_amdgcn_s_memtime() - t_pub;
#endif
        if (!ok) {
          if (lane == 0) { atomicOr(c.err, 4); s_abort = 1; }
        } else if (lane == 0) {
          s_g[0] = a_mn < 0 ? a_mn : 0;  // the accumulators start at 0 (interpod_affinity.go:129-131)
          s_g[1] = a_mx > 0 ? a_mx : 0;
          s_g[2] = a_smx; s_g[3] = a_hz;
          s_g[4] = zmax;
          if (AUX) s_g[8] = azmax;  // (over every domain: zeros included, as passa_reduce)
        }
      } else if (pend_j >= 0) {
        // the previous pod's deferred commit, inside this exchange window
        PgX Xp;
        Xp.base = xrec(pend_pod);
        const PgHdr Hp = pg_hdr_u(Xp.hdr());
        pg_sections(Hp, Xp.so);
#ifdef KSIM_STAMPS
        const uint64_t tc0 = __builtin_amdgcn_s_memtime();
#endif
        pg_commit_row(c, g, L, Xp, Hp, pend_j, lo + pend_j);
#ifdef KSIM_STAMPS
        cm_acc += __builtin_amdgcn_s_memtime() - tc0;
        cm_n += 1;
#endif
        pend_j = -1;
      }
      __syncthreads();
      if (s_abort) { stop_pod = pod; break; }
      const int64_t gmn = s_g[0], gmx = s_g[1], gsmx = s_g[2], ghz = s_g[3], gzm = s_g[4];
      const int64_t gamx = AUX ? s_g[5] : 0, gatot = AUX ? s_g[6] : 0, gahz = AUX ? s_g[7] : 0, gazm = AUX ? s_g[8] : 0;
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        if (!cur[k].fit) continue;
        if (ap >= 0) {  // (aux_add's)
          const int32_t d = L.dom[(int64_t)g.A.aux_key * chunk + k * PG_RT + rt];
          const int64_t ds = d >= 0 ? s_gaz[d] : 0;
          cur[k].sc = (int64_t)((uint64_t)cur[k].sc + (uint64_t)g.A.aux_w * (uint64_t)ksim_aux_score(g.A.aux_kind, cur[k].acnt, d, ds,
                                                                                                   gamx, gatot, gahz != 0, gazm));
        }
        if (ipa)
          cur[k].sc = (int64_t)((uint64_t)cur[k].sc +
                                (uint64_t)c.w[KSIM_W_INTERPOD_AFFINITY] * (uint64_t)ksim_interpod_score(cur[k].raw, gmn, gmx));
        if (sp >= 0)
          cur[k].sc = (int64_t)((uint64_t)cur[k].sc +
                                (uint64_t)c.w[KSIM_W_SELECTOR_SPREAD] *
                                    (uint64_t)ksim_spread_score(cur[k].cnt, gsmx, ghz != 0, cur[k].zz,
                                                                cur[k].zz >= 0 ? s_gz[cur[k].zz] : 0, gzm));
      }
    }
    if (aon && ap < 0) {  // serviceAntiAffinity of a pod no service selects: 10 on a labelled row (no pass A)
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        if (!cur[k].fit) continue;
        const int32_t d = L.dom[(int64_t)g.A.aux_key * chunk + k * PG_RT + rt];
        cur[k].sc = (int64_t)((uint64_t)cur[k].sc + (uint64_t)g.A.aux_w * (uint64_t)ksim_aux_score(g.A.aux_kind, 0, d, 0, 0, 0, false, 0));
      }
    }
    if (pend_j >= 0) {  // the previous pod's deferred commit, when no pass-A window took it
      PgX Xp;
      Xp.base = xrec(pend_pod);
      const PgHdr Hp = pg_hdr_u(Xp.hdr());
      pg_sections(Hp, Xp.so);
#ifdef KSIM_STAMPS
      const uint64_t tc0 = __builtin_amdgcn_s_memtime();
#endif
      pg_commit_row(c, g, L, Xp, Hp, pend_j, lo + pend_j);
#ifdef KSIM_STAMPS
      cm_acc += __builtin_amdgcn_s_memtime() - tc0;
      cm_n += 1;
#endif
      pend_j = -1;
    }
    if (wv == 4 && L.hd) {
      // the dense hypothesis deltas: pod p-1's entries out, pod p's in (read by the E1 waves in this
      // pod's decision window; pod p-1's readers finished before its decision barrier)
      if (pod > c.first) {
        PgX Xq;
        Xq.base = xrec(pod - 1);
        const PgHdr Hq = pg_hdr_u(Xq.hdr());
        pg_sections(Hq, Xq.so);
        const int2* mp = Xq.sec<int2>(PGS_MP);
        for (int32_t x = lane; x < Hq.n_mp; x += 64) L.hd[mp[x].x] = 0;
        const PgCar* cr = Xq.sec<PgCar>(PGS_CAR);
        for (int32_t x = lane; x < Hq.n_car; x += 64) { L.hc[cr[x].term] = 0; L.hk[cr[x].term] = 0; }
      }
      const int2* mp = X.sec<int2>(PGS_MP);
      for (int32_t x = lane; x < H.n_mp; x += 64) L.hd[mp[x].x] = mp[x].y + 1;
      const PgCar* cr = X.sec<PgCar>(PGS_CAR);
      for (int32_t x = lane; x < H.n_car; x += 64) { L.hc[cr[x].term] = cr[x].amount; L.hk[cr[x].term] = cr[x].key + 1; }
    }
    PG_STAMP(1);

    // ---- per reduce class (max, count) and fit count of this workgroup's rows ----
    int32_t nf = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) nf += __popcll(__ballot(cur[k].fit));
    if (lane == 0) s_fit[wv] = nf;
    for (int q = 0; q < K; ++q) {
      int32_t v = -1;
#pragma unroll
      for (int k = 0; k < NPT; ++k)
        if (cur[k].fit && cur[k].cl == q && (int32_t)cur[k].sc > v) v = (int32_t)cur[k].sc;
      const int32_t wm = ksimw::max_i32(v);
      int32_t cn = 0;
#pragma unroll
      for (int k = 0; k < NPT; ++k) cn += __popcll(__ballot(cur[k].fit && cur[k].cl == q && (int32_t)cur[k].sc == wm));
      if (lane == 0) { s_mx[wv][q] = wm; s_cn[wv][q] = wm < 0 ? 0 : cn; }
    }
    __syncthreads();
    PG_STAMP(2);

    // ---- wave 0: publish, sweep, decide; row threads: pod p+1 on every row, E0 and E1 ----
    PgEv n0[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) n0[k] = PgEv{0, 0, 0, 0, -1, 0, false};
    if (wv == 0) {
      if (lane < K) {
        int32_t m = -1, nn = 0, f = 0;
#pragma unroll
        for (int w = 0; w < PG2_NW; ++w) {
          f += s_fit[w];
          if (!s_cn[w][lane]) continue;
          if (s_mx[w][lane] > m) { m = s_mx[w][lane]; nn = s_cn[w][lane]; }
          else if (s_mx[w][lane] == m) nn += s_cn[w][lane];
        }
        const uint64_t v = ((uint64_t)tag << 56) | (lane == 0 ? ((uint64_t)f << 44) : 0) | ((uint64_t)nn << 32) |
                           (uint64_t)(uint32_t)m;
        pg_store(cls_at(g.gran, slot, lane, blockIdx.x), v);
      }
#ifdef KSIM_STAMPS
      t_pub = __builtin_amdgcn_s_memtime();
#endif
      // the decision's per-class map values (lane q = reduce class q)
      int64_t tv_l = 0, av_l = 0, ad_l = 0;
      if (lane < K) {
        tv_l = X.tv(K > 1 ? lane / k2 : 0);
        av_l = X.av(K > 1 ? lane % k2 : 0);
        ad_l = X.ad(K > 1 ? lane % k2 : 0);
      }
      int mode = 0, blk = -1, rank = 0;
      uint32_t win = 0;
      int32_t tgt_l = -2;  // lane q: class q's maximum if q wins
      // the workgroup holding the ix-th match from the top (lane-major workgroup order: lane l
      // holds l, l + 64, ...; name rank grows with the workgroup index), bm = matches per workgroup
      auto locate = [&](const int32_t (&bm)[MB], int64_t ix) {
        // matches in workgroups above b = (lanes above, same m) + (every lane, higher m)
        int64_t above = 0;
        int found = -1, rk = 0;
#pragma unroll
        for (int m = MB - 1; m >= 0; --m) {
        if (found < 0 && 64 * m < G) {
          const int32_t pre = ksimw::prefix_incl_i32(bm[m]);
          const int32_t tot = __builtin_amdgcn_readlane(pre, 63);
          const int64_t ab = above + (int64_t)(tot - pre);
          const bool hit = bm[m] > 0 && ix >= ab && ix < ab + bm[m];
          const uint64_t hb = __ballot(hit);
          if (hb) {
            const int src = __builtin_ffsll((long long)hb) - 1;
            found = src + 64 * m;
            rk = (int)__builtin_amdgcn_readlane((int32_t)(ix - ab), src);
          }
          above += tot;
        }
        }
        if (found < 0) { mode = -1; if (lane == 0) atomicOr(c.err, 2); }
        blk = found;
        rank = rk;
      };
      if (K == 1) {
        // one reduce class (no TaintToleration / NodeAffinity spread among the fit nodes): the
        // class maximum is the best total, and only granule 0 of each workgroup is read
        uint64_t gv0[MB];
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool ok = false;
        for (;;) {
          bool mine = true;
#pragma unroll
          for (int m = 0; m < MB; ++m) {
            const int b = lane + 64 * m;
            gv0[m] = b < G ? pg_load(cls_at(g.gran, slot, 0, b)) : ((uint64_t)tag << 56);
            mine &= gtag(gv0[m]) == tag;
          }
          if (__all(mine)) { ok = true; break; }
          if (__builtin_amdgcn_s_memrealtime() - t0 > g.spin_ticks) break;
          __builtin_amdgcn_s_sleep(1);
        }
#ifdef KSIM_STAMPS
        cs_acc += __builtin_amdgcn_s_memtime() - t_pub;
        if (blockIdx.x == 0 && tid == 0) PG_STAMP(7);
#endif
        if (!ok) {
          mode = -1;
          if (lane == 0) atomicOr(c.err, 4);
        } else {
          int32_t f = 0, mm = -1, cc = 0;
#pragma unroll
          for (int m = 0; m < MB; ++m) {
            if (lane + 64 * m >= G) continue;
            f += gfit(gv0[m]);
            const int32_t cn = gcnt(gv0[m]), sc0 = gscore(gv0[m]);
            if (!cn) continue;
            if (sc0 > mm) { mm = sc0; cc = cn; }
            else if (sc0 == mm) cc += cn;
          }
          const int32_t F = ksimw::sum_i32(f);
          if (F > 0) {
            mode = 1;
            int64_t ix = 0;
            int32_t M0 = -1;
            if (F > 1) {  // generic_scheduler.go:153-156: a single fit skips selectHost
              mode = 2;
              M0 = ksimw::max_i32(cc ? mm : -1);
              const int32_t C = ksimw::sum_i32((cc && mm == M0) ? cc : 0);
              win = 1;
              tgt_l = lane == 0 ? M0 : -2;
              ix = (counter >> 32) ? (int64_t)(counter % (uint64_t)C) : (int64_t)((uint32_t)counter % (uint32_t)C);
              counter += 1;  // generic_scheduler.go:192-195
            }
            int32_t bm[MB];
#pragma unroll
            for (int m = 0; m < MB; ++m) {
              int32_t sb = 0;
              if (lane + 64 * m < G)
                sb = mode == 1 ? gfit(gv0[m]) : ((gcnt(gv0[m]) && gscore(gv0[m]) == M0) ? gcnt(gv0[m]) : 0);
              bm[m] = sb;
            }
            locate(bm, ix);
          }
        }
      } else {
        uint64_t gv[KSIM_MAX_RCLASS][MB];
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool ok = false;
        for (;;) {
          bool mine = true;
#pragma unroll
          for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
#pragma unroll
            for (int m = 0; m < MB; ++m) {
              const int b = lane + 64 * m;
              gv[q][m] = (q < K && b < G) ? pg_load(cls_at(g.gran, slot, q, b)) : ((uint64_t)tag << 56);
              mine &= gtag(gv[q][m]) == tag;
            }
          }
          if (__all(mine)) { ok = true; break; }
          if (__builtin_amdgcn_s_memrealtime() - t0 > g.spin_ticks) break;
          __builtin_amdgcn_s_sleep(1);
        }
#ifdef KSIM_STAMPS
        cs_acc += __builtin_amdgcn_s_memtime() - t_pub;
        if (blockIdx.x == 0 && tid == 0) PG_STAMP(7);
#endif
        if (!ok) {
          mode = -1;
          if (lane == 0) atomicOr(c.err, 4);
        } else {
          int32_t F = 0;
          int32_t mq_l = -1, cq_l = 0;  // lane q: class q's global maximum and its count
          int32_t f = 0;
#pragma unroll
          for (int m = 0; m < MB; ++m) f += (lane + 64 * m < G) ? gfit(gv[0][m]) : 0;
          F = ksimw::sum_i32(f);
#pragma unroll
          for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
            if (q < K) {
              int32_t mm = -1, cc = 0;
#pragma unroll
              for (int m = 0; m < MB; ++m) {
                if (lane + 64 * m >= G) continue;
                const int32_t cn = gcnt(gv[q][m]), s = gscore(gv[q][m]);
                if (!cn) continue;
                if (s > mm) { mm = s; cc = cn; }
                else if (s == mm) cc += cn;
              }
              const int32_t Mq = ksimw::max_i32(cc ? mm : -1);
              const int32_t Cq = ksimw::sum_i32((cc && mm == Mq) ? cc : 0);
              mq_l = lane == q ? Mq : mq_l;
              cq_l = lane == q ? Cq : cq_l;
            }
          }
#ifdef KSIM_STAMPS
          if (blockIdx.x == 0 && tid == 0) PG_STAMP(11);
#endif
          if (F > 0) {
            mode = 1;
            int64_t ix = 0;
            if (F > 1) {  // generic_scheduler.go:153-156: a single fit skips selectHost
              mode = 2;
              // lane q = reduce class q: NormalizeReduce over the filtered set, weighted totals
              // (reduce.go:29-64, generic_scheduler.go:632-639), the best total and its classes
              const bool live = lane < K && cq_l != 0;
              int64_t mxT = 0, mxA = 0;
              // K <= 16: the class lanes are one DPP row
              if (k1 > 1 || c.w[KSIM_W_TAINT_TOLERATION]) mxT = ksimw::max16_i64(live ? tv_l : 0);
              if (k2 > 1 || c.w[KSIM_W_NODE_AFFINITY]) mxA = ksimw::max16_i64(live ? av_l : 0);
              uint64_t t = (uint64_t)(int64_t)mq_l + (uint64_t)ad_l;
              if (c.w[KSIM_W_TAINT_TOLERATION]) t += (uint64_t)c.w[KSIM_W_TAINT_TOLERATION] * (uint64_t)ksim_norm(tv_l, mxT, true);
              if (c.w[KSIM_W_NODE_AFFINITY]) t += (uint64_t)c.w[KSIM_W_NODE_AFFINITY] * (uint64_t)ksim_norm(av_l, mxA, false);
              const int64_t tot = live ? (int64_t)t : INT64_MIN;
              const int64_t best = ksimw::max16_i64(tot);
              const uint64_t wbm = __ballot(live && tot == best);
              win = (uint32_t)wbm;
              const int32_t C = ksimw::sum16_i32(((wbm >> lane) & 1ull) ? cq_l : 0);
              tgt_l = ((wbm >> lane) & 1ull) ? mq_l : -2;
              ix = (counter >> 32) ? (int64_t)(counter % (uint64_t)C) : (int64_t)((uint32_t)counter % (uint32_t)C);
              counter += 1;  // generic_scheduler.go:192-195
            }
            // locate the workgroup holding the ix-th match from the top (lane-major workgroup order:
            // lane l holds l, l + 64, ...; name rank grows with the workgroup index)
            int32_t bm[MB];
#pragma unroll
            for (int m = 0; m < MB; ++m) {
              const int b = lane + 64 * m;
              int32_t s = 0;
              if (b < G) {
                if (mode == 1) {
                  s = gfit(gv[0][m]);
                } else {
#pragma unroll
                  for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
                    if (q < K && ((win >> q) & 1u)) {
                      const int32_t Mq = __builtin_amdgcn_readlane(mq_l, q);
                      if (gcnt(gv[q][m]) && gscore(gv[q][m]) == Mq) s += gcnt(gv[q][m]);
                    }
                  }
                }
              }
              bm[m] = s;
            }
            locate(bm, ix);
          }
        }
      }
#ifdef KSIM_STAMPS
      if (blockIdx.x == 0 && tid == 0) PG_STAMP(12);
#endif
      if (lane < KSIM_MAX_RCLASS) s_tgt[lane] = tgt_l;
      if (lane == 0) { s_mode = mode; s_blk = blk; s_rank = rank; s_win = win; s_node = -1; }
    } else if (pf) {
      const uint4* src = reinterpret_cast<const uint4*>(g.rec + (pod + 2 - c.first) * (int64_t)g.d.rec_stride);
      uint4* dst = reinterpret_cast<uint4*>(xrec(pod + 2));
      for (int32_t x = lane; x < g.d.rec_stride / 16; x += 64) dst[x] = src[x];
    } else if ((rowt || hypt) && has_next) {
#ifdef KSIM_STAMPS
      const uint64_t te0 = __builtin_amdgcn_s_memtime();
      uint64_t* sa = (tid == 64 || tid == 320) ? ev_sa : nullptr;
#else
      uint64_t* sa = nullptr;
#endif
      PgX X1;
      X1.base = xrec(pod + 1);
      const PgHdr H1 = pg_hdr_u(X1.hdr());
      pg_sections(H1, X1.so);
      const ksim_pod P1 = pg_pod_u(X1.pod());
      const PgHyp y{&X, &H};
      if (rowt) {
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int32_t j = k * PG_RT + rt;
          if (j < nrows) n0[k] = pg_eval<false, AUX>(c, g, L, X1, P1, H1, j, lo + j, y, P, k == 0 ? sa : nullptr);
        }
      } else if (!(H.fl & PGF_NOHYP) && !c.no_commit) {
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int32_t j = k * PG_RT + rt;
          if (j < nrows) ev1[j] = pg_eval<true, AUX>(c, g, L, X1, P1, H1, j, lo + j, y, P, k == 0 ? sa : nullptr);
        }
      }
#ifdef KSIM_STAMPS
      if (tid == 64) ev_acc += __builtin_amdgcn_s_memtime() - te0;
      if (tid == 320) ev_acc1 += __builtin_amdgcn_s_memtime() - te0;
#endif
    }
    __syncthreads();
    PG_STAMP(3);
    const int mode = s_mode;
    if (mode < 0) { stop_pod = pod; break; }  // uniform: every workgroup reached the same verdict

    // ---- FitError: every workgroup adds its rows' reasons; nothing committed ----
    if (mode == 0) {
      if (c.collect && c.out_reasons && rowt) {
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          if (!__ballot(cur[k].rmk != 0)) continue;
          for (int r = 0; r < KSIM_NREASONS; ++r) {
            const int32_t nr = __popcll(__ballot((cur[k].rmk >> r) & 1u));
            if (lane == 0 && nr) atomicAdd(&c.out_reasons[pod * KSIM_NREASONS + r], nr);
          }
        }
      }
      if (blockIdx.x == 0 && tid == 0) c.out_node[pod] = -1;
#pragma unroll
      for (int k = 0; k < NPT; ++k) cur[k] = n0[k];
      continue;
    }

    // ---- the owner picks the row (the rank-th match from the top, selectHost's order) ----
    const bool owner = s_blk == (int)blockIdx.x;
    const bool shared = (H.fl & PGF_SHARED) != 0;
    const bool aff_commit = (H.fl & PGF_AFF) && !c.no_commit;
    int ksel = -1;
    if (owner) {
      const uint32_t win = s_win;
      const int32_t rr = s_rank;
      bool mt[NPT];
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        mt[k] = rowt && cur[k].fit && (mode == 1 || (((win >> cur[k].cl) & 1u) && (int32_t)cur[k].sc == s_tgt[cur[k].cl]));
        const uint64_t bl = __ballot(mt[k]);
        if (lane == 0 && rowt) s_bal[k][wv - 1] = bl;
      }
      __syncthreads();
      int32_t above = 0;
#pragma unroll
      for (int k = NPT - 1; k >= 0; --k) {
        int32_t up = 0;
#pragma unroll
        for (int w = PG_RW - 1; w >= 0; --w)
          if (rowt && w > wv - 1) up += __popcll(s_bal[k][w]);
        const int32_t mine = rowt ? __popcll((s_bal[k][wv - 1] >> lane) >> 1) : 0;
        if (mt[k] && above + up + mine == rr) ksel = k;
#pragma unroll
        for (int w = 0; w < PG_RW; ++w) above += __popcll(s_bal[k][w]);
      }
      if (rr >= above) {  // uniform in the owner workgroup
        if (tid == 0) atomicOr(c.err, 2);
        break;
      }
    }
    int32_t jsel = -1;
    if (ksel >= 0) {
      jsel = ksel * PG_RT + rt;
      const int64_t w = lo + jsel;
      c.out_node[pod] = (int32_t)w;
      if (shared) {
        s_node = w;
        pg_store(g.gran + PG_COMMIT_OFF + slot, ((uint64_t)tag << 56) | (uint64_t)w);
      }
    }
    PG_STAMP(4);
    if (!(H.fl & PGF_NOHYP) || c.no_commit) {
      // the hypothesis holds: every row takes E0, the chosen row E1, its commit is deferred
#pragma unroll
      for (int k = 0; k < NPT; ++k) cur[k] = (k == ksel && !c.no_commit) ? ev1[k * PG_RT + rt] : n0[k];
      if (jsel >= 0 && !c.no_commit) {
        pend_j = jsel;
        pend_pod = pod;
      }
      PG_STAMP(5);
      continue;
    }
    // ---- no hypothesis: commit now, shared domains in every workgroup, re-evaluate pod p+1 ----
    if (jsel >= 0) pg_commit_row(c, g, L, X, H, jsel, lo + jsel);
    if (shared && aff_commit) {
      if (!owner && tid == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint64_t v;
        while (gtag(v = pg_load(g.gran + PG_COMMIT_OFF + slot)) != tag) {
          if (__builtin_amdgcn_s_memrealtime() - t0 > g.spin_ticks) { atomicOr(c.err, 4); s_abort = 1; break; }
          __builtin_amdgcn_s_sleep(1);
        }
        s_node = (int64_t)(v & M56);
      }
      __syncthreads();
      if (s_abort) { stop_pod = pod; break; }
      const int64_t w = s_node;
      const int2* mp = X.sec<int2>(PGS_MP);
      const PgCar* cr = X.sec<PgCar>(PGS_CAR);
      const int32_t nm = H.n_mp, ncr = H.n_car;
      for (int32_t x = tid; x < nm + ncr; x += PG2_BS) {
        const int32_t key = x < nm ? mp[x].y : cr[x - nm].key;
        s_dw[x] = g.A.dom[(int64_t)key * n + w];
      }
      __syncthreads();
      for (int32_t yy = tid; yy < (nm + ncr) * nrows; yy += PG2_BS) {
        const int32_t x = yy / nrows, j = yy - x * nrows;
        const int32_t dw = s_dw[x];
        if (dw < 0) continue;
        if (x < nm) {
          if (L.dom[(int64_t)mp[x].y * chunk + j] == dw) L.cnt[(int64_t)mp[x].x * chunk + j] += 1;
        } else {
          const PgCar& k = cr[x - nm];
          if (L.dom[(int64_t)k.key * chunk + j] == dw)
            atomicAdd(reinterpret_cast<unsigned long long*>(&L.car[(int64_t)k.term * chunk + j]), (unsigned long long)k.amount);
        }
      }
    }
    __syncthreads();
    if (has_next && rowt) {
      PgX X1;
      X1.base = xrec(pod + 1);
      const PgHdr H1 = pg_hdr_u(X1.hdr());
      pg_sections(H1, X1.so);
      const ksim_pod P1 = pg_pod_u(X1.pod());
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int32_t j = k * PG_RT + rt;
        // shared domains may have changed any row; otherwise only the chosen one
        if (j < nrows && (shared || k == ksel)) cur[k] = pg_eval<false, AUX>(c, g, L, X1, P1, H1, j, lo + j, PgHyp{}, P1);
        else cur[k] = n0[k];
      }
    }
    PG_STAMP(5);
  }
  if (pend_j >= 0) {  // the last deferred commit
    PgX Xp;
    Xp.base = xrec(pend_pod);
    const PgHdr Hp = pg_hdr_u(Xp.hdr());
    pg_sections(Hp, Xp.so);
    pg_commit_row(c, g, L, Xp, Hp, pend_j, lo + pend_j);
  }
  pg_write_back(c, g, L, lo, nrows, chunk, tid, blockDim.x);
  if (tid == 0 && stop_pod < c.end) atomicMin((unsigned long long*)c.cursor, (unsigned long long)stop_pod);
#ifdef KSIM_STAMPS
  // the spread over workgroups: max and (as ~max of ~) min of pass-A exchange, classes, decide
  // window, pass-A local, and of the row evaluations
  if (tid == 0) {
    const int ks[4] = {1, 2, 3, 6};
    for (int x = 0; x < 4; ++x) {
      atomicMax((unsigned long long*)&c.dbg[16 + 2 * x], (unsigned long long)st_acc[ks[x]]);
      atomicMax((unsigned long long*)&c.dbg[17 + 2 * x], (unsigned long long)~st_acc[ks[x]]);
    }
  }
  if (cm_n) {
    atomicAdd((unsigned long long*)&c.dbg[32], (unsigned long long)cm_acc);
    atomicAdd((unsigned long long*)&c.dbg[36], (unsigned long long)cm_n);
  }
  if (tid == 0) {
    atomicAdd((unsigned long long*)&c.dbg[33], (unsigned long long)ps_acc);
    atomicAdd((unsigned long long*)&c.dbg[34], (unsigned long long)pr_acc);
    atomicAdd((unsigned long long*)&c.dbg[35], (unsigned long long)cs_acc);
  }
  if (tid == 64 || tid == 320)
    for (int x = 0; x < 6; ++x) atomicAdd((unsigned long long*)&c.dbg[26 + x], (unsigned long long)ev_sa[x]);
  if (tid == 64) {
    atomicMax((unsigned long long*)&c.dbg[24], (unsigned long long)ev_acc);
    atomicMax((unsigned long long*)&c.dbg[25], (unsigned long long)~ev_acc);
  }
  if (tid == 320) {
    atomicMax((unsigned long long*)&c.dbg[14], (unsigned long long)ev_acc1);
    atomicMax((unsigned long long*)&c.dbg[15], (unsigned long long)~ev_acc1);
  }
#endif
  if (blockIdx.x == 0 && tid == 0) {
    *c.counter = counter;
    (void)0;  // the cursor: c.end preset by the host, lowered below by an aborting workgroup
#ifdef KSIM_STAMPS
    for (int k = 0; k < 16; ++k) c.dbg[k] += st_acc[k];
#endif
  }
}

extern "C" size_t ksim_pgen_gran_bytes(void) { return (size_t)PG_GRAN_WORDS * sizeof(uint64_t); }
extern "C" int ksim_pgen_max_zones(void) { return PG_MAXZ; }
extern "C" int ksim_pgen_max_aux_domains(void) { return PG_MAXAD; }
extern "C" size_t ksim_pgen_lds_budget(void) { return PG_LDS_BUDGET; }

// LDS layout for `chunk` rows per workgroup (the kernel rebuilds its pointers from off[]).
extern "C" size_t ksim_pgen_plan(int64_t chunk, const PgDims* d, uint32_t* off) {
  auto al = [](size_t b) { return (b + 15) & ~(size_t)15; };
  const size_t C = (size_t)chunk;
  size_t o = 0;
  auto put = [&](int k, size_t bytes) { off[k] = (uint32_t)o; o += al(bytes); };
  put(PGO_AC, C * 8); put(PGO_AM, C * 8); put(PGO_RC, C * 8); put(PGO_RM, C * 8); put(PGO_ZC, C * 8); put(PGO_ZM, C * 8);
  put(PGO_AL, C * 4); put(PGO_CT, C * 4); put(PGO_FL, C * 4); put(PGO_LS, C * 4); put(PGO_TS, C * 4);
  put(PGO_SC, C * 4); put(PGO_CL, C);
  put(PGO_ST, (size_t)d->n_st * C * 2);
  put(PGO_VC, d->vcap ? C * 4 : 0); put(PGO_VH, d->vcap ? C * 6 : 0); put(PGO_VS, (size_t)d->vslots * C * 8);
  put(PGO_PC, d->pslots ? C * 4 : 0); put(PGO_PK, (size_t)d->pslots * C * 8);
  put(PGO_DOM, (size_t)d->n_keys * C * 4); put(PGO_CNT, (size_t)d->n_pair * C * 4); put(PGO_CAR, (size_t)d->n_carry * C * 8);
  put(PGO_X0, (size_t)d->rec_stride); put(PGO_X1, (size_t)d->rec_stride);
  put(PGO_X2, d->hyp ? (size_t)d->rec_stride : 0); put(PGO_X3, d->hyp ? (size_t)d->rec_stride : 0);
  put(PGO_E1, d->hyp ? C * PG_EV_BYTES : 0);
  put(PGO_HD, d->hdense ? (size_t)d->n_pair * 4 : 0);
  put(PGO_HC, d->hdense ? (size_t)d->n_carry * 8 : 0);
  put(PGO_HK, d->hdense ? (size_t)d->n_carry * 4 : 0);
  return o;
}

template <int NPT, int MB>
static hipError_t launch_pgen(const KsimCtx* c, const PGenArgs* g, int grid, size_t lds, hipStream_t s) {
  hipError_t e = ksim_check_coresident(ksim_pgen_kernel<NPT, MB>, grid, PG_BS, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((ksim_pgen_kernel<NPT, MB>), dim3(grid), dim3(PG_BS), lds, s, *c, *g);
  return hipGetLastError();
}

extern "C" hipError_t ksim_launch_pgen(const KsimCtx* c, const PGenArgs* g, int grid, int npt, size_t lds, hipStream_t s) {
  if (grid <= 0 || grid > PG_MAXG || g->d.rec_stride % 16 || g->d.rec_stride > PG_REC_MAX || lds > PG_LDS_BUDGET ||
      (int64_t)grid * c->chunk < c->n || c->chunk > (int64_t)npt * PG_BS)
    return hipErrorInvalidValue;
  if (grid <= 64) {
    switch (npt) {
      case 1: return launch_pgen<1, 1>(c, g, grid, lds, s);
      case 2: return launch_pgen<2, 1>(c, g, grid, lds, s);
      default: return launch_pgen<4, 1>(c, g, grid, lds, s);
    }
  }
  switch (npt) {
    case 1: return launch_pgen<1, 4>(c, g, grid, lds, s);
    case 2: return launch_pgen<2, 4>(c, g, grid, lds, s);
    default: return launch_pgen<4, 4>(c, g, grid, lds, s);
  }
}

template <int NPT, int MB, bool AUX>
static hipError_t launch_pgen2(const KsimCtx* c, const PGenArgs* g, int grid, size_t lds, hipStream_t s) {
  hipError_t e = ksim_check_coresident(ksim_pgen2_kernel<NPT, MB, AUX>, grid, PG2_BS, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((ksim_pgen2_kernel<NPT, MB, AUX>), dim3(grid), dim3(PG2_BS), lds, s, *c, *g);
  return hipGetLastError();
}

extern "C" hipError_t ksim_launch_pgen2(const KsimCtx* c, const PGenArgs* g, int grid, int npt, size_t lds, hipStream_t s) {
  if (grid <= 0 || grid > PG_MAXG || g->d.rec_stride % 16 || g->d.rec_stride > PG_REC_MAX || lds > PG_LDS_BUDGET ||
      (int64_t)grid * c->chunk < c->n || c->chunk > (int64_t)npt * PG_RT || (npt != 1 && npt != 2 && npt != 4) || !g->d.hyp ||
      grid > 64)
    return hipErrorInvalidValue;
  // the auxiliary priority's instantiation only for handles with its tables
  const bool aux = g->has_aff && g->A.aux_pair && g->A.aux_w != 0 && !c->no_prio;
  switch (npt) {  // one granule per lane in the sweeps (grid <= 64; larger grids take the single form)
    case 1: return aux ? launch_pgen2<1, 1, true>(c, g, grid, lds, s) : launch_pgen2<1, 1, false>(c, g, grid, lds, s);
    case 2: return aux ? launch_pgen2<2, 1, true>(c, g, grid, lds, s) : launch_pgen2<2, 1, false>(c, g, grid, lds, s);
    default: return aux ? launch_pgen2<4, 1, true>(c, g, grid, lds, s) : launch_pgen2<4, 1, false>(c, g, grid, lds, s);
  }
}

extern "C" hipError_t ksim_pgen_pack(const KsimCtx* c, const PGenArgs* g, hipStream_t s) {
  const int64_t count = c->end - c->first;
  if (count <= 0) return hipSuccess;
  const int grid = (int)std::min<int64_t>(count, 8192);
  hipLaunchKernelGGL(ksim_pgen_pack_kernel, dim3(grid), dim3(64), 0, s, *c, *g);
  return hipGetLastError();
}
