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
//      node_info.go:318-341: LDS row, HBM side columns, host ports, volume mounts) and applies the
//      pod's affinity counts to its rows; when those counts live in shared topology domains (zones,
//      "anywhere"), the owner publishes the node in a tagged commit word and EVERY workgroup applies
//      the counts to its own rows of that domain (one more exchange for such pods only).
//
// What a row's evaluation reads sits in LDS, so it is a chain of LDS round trips rather than of
// dependent HBM / L2 loads: the 60-byte resource row, the label / taint set ids, one static 16-bit
// word per (pod class, row) built at launch (selector, NoSchedule / NoExecute taints, service
// affinity verdicts, TaintToleration / NodeAffinity reduce classes), the row's first volume mounts
// and its per-MaxPD-filter mounted-volume counts.
//
// Affinity counts in "row" form: for counted pair c (selector, topology key) and node i the kernel
// keeps cnt_row[c][i] = the pair's count in i's domain of the key (0 when i lacks the key), and
// car_row[e][i] likewise for carried terms.  Placing a pod on node w adds to the rows of every node
// in w's domain — each workgroup updates its own rows, so these arrays are private to their owner
// (no cross-workgroup coherence) while shared domains stay consistent by replication.  The host
// builds them from the canonical per-domain counts before the launch and folds them back after
// (ksim_pgen_rows).  Volume slots and host ports are only touched by the owner of a row, so their
// HBM columns stay authoritative (the LDS copy mirrors them).
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
#define PG_RA (4 + PG_MAXZ)  // words of a pass-A record
#define PG_MB (PG_MAXG / 64)
// exchange buffer: pass-A records, class granules, then one commit word per slot
#define PG_COMMIT_OFF ((int64_t)PG_NSLOT * (PG_RA + KSIM_MAX_RCLASS) * PG_MAXG)
#define PG_GRAN_WORDS (PG_COMMIT_OFF + PG_NSLOT)
#define PG_LDS_BUDGET (150 * 1024)
#define PG_VS_MAX 8

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

__device__ __forceinline__ int64_t wmax64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t t = __shfl_xor(v, o, 64);
    v = t > v ? t : v;
  }
  return v;
}
__device__ __forceinline__ int64_t wmin64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t t = __shfl_xor(v, o, 64);
    v = t < v ? t : v;
  }
  return v;
}
__device__ __forceinline__ int64_t wsum64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// The workgroup's LDS image (struct of arrays, `chunk` entries each; ksim_pgen_plan sizes it).
struct PgLds {
  int64_t *ac, *am, *rc, *rm, *zc, *zm;  // the 60-byte resource row
  int32_t *al, *ct;
  uint32_t* fl;
  int32_t *ls, *ts;                      // label / taint set ids
  int32_t* sc;                           // this pod's total score, -1: does not fit
  uint8_t* cl;                           // its reduce class
  int32_t* vc;                           // volume mounts of the row (slot_count)
  uint16_t* vh;                          // [3][chunk] mounted keys counted by the EBS / GCE PD / Azure filters
  uint64_t* vs;                          // [vs][chunk] the row's first vs slots
  uint16_t* st;                          // [classes][chunk] static words, or null
  int64_t chunk;
  int32_t nvs;
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

// Slot s of row j (node i): LDS for the first nvs, HBM beyond.
__device__ __forceinline__ uint64_t pg_slot(const KsimVol& V, const PgLds& L, int32_t j, int64_t i, int32_t s) {
  return s < L.nvs ? L.vs[(int64_t)s * L.chunk + j] : V.slots[(int64_t)s * V.n + i];
}

__device__ __forceinline__ int32_t pg_vol_find(const KsimVol& V, const PgLds& L, int32_t j, int64_t i, int32_t cnt,
                                               int32_t key) {
  for (int32_t s = 0; s < cnt; ++s)
    if ((int32_t)(pg_slot(V, L, j, i, s) >> 32) == key) return s;
  return -1;
}

// NoDiskConflict (predicates.go:276-285 over isVolumeConflict :220-265), as ksim_disk_conflict.
__device__ __noinline__ uint32_t pg_disk_conflict(const KsimVol& V, const PgLds& L, int32_t vclass, int32_t j,
                                                  int64_t i) {
  const int32_t* vc = V.vc + 2 * (int64_t)(vclass - 1);
  const int32_t cnt = L.vc[j];
  if (!cnt) return 0;
  for (int32_t r = vc[0], e = vc[0] + vc[1]; r < e; ++r) {
    const ksim_vol_ref ref = V.refs[r];
    if (!(ref.flags & (KSIM_VOL_CONFLICT_ANY | KSIM_VOL_CONFLICT_RW))) continue;
    const int32_t s = pg_vol_find(V, L, j, i, cnt, ref.key);
    if (s < 0) continue;
    const uint64_t w = pg_slot(V, L, j, i, s);
    const uint32_t rw = (uint32_t)(w & 0x7FFu), ro = (uint32_t)((w >> 11) & 0x7FFu);
    if ((ref.flags & KSIM_VOL_CONFLICT_ANY) ? (rw + ro > 0) : (rw > 0)) return 1u << KSIM_R_DISK_CONFLICT;
  }
  return 0;
}

// MaxEBS / MaxGCEPD / MaxAzureDiskVolumeCount (predicates.go:415-456), as ksim_max_volumes: the
// row's mounted keys each filter counts (LDS) plus the pod's new keys not mounted yet.
__device__ __noinline__ uint32_t pg_max_volumes(const KsimVol& V, const PgLds& L, int32_t vclass, int32_t j, int64_t i,
                                                uint32_t which) {
  const uint32_t want = V.vc_filter[vclass - 1] & which;
  if (!want) return 0;
  const int32_t* vc = V.vc + 2 * (int64_t)(vclass - 1);
  const int32_t cnt = L.vc[j];
  for (int t = 0; t < 3; ++t) {
    const uint32_t f = 1u << t;
    if (!(want & f)) continue;
    int32_t add = 0;
    for (int32_t r = vc[0], e = vc[0] + vc[1]; r < e; ++r) {
      const ksim_vol_ref ref = V.refs[r];
      if ((ref.flags & KSIM_VOL_NEW) && (V.key_filter[ref.key] & f) && pg_vol_find(V, L, j, i, cnt, ref.key) < 0) ++add;
    }
    if ((int32_t)L.vh[(int64_t)t * L.chunk + j] + add > V.max_vols[t]) return 1u << KSIM_R_MAX_VOLUME_COUNT;
  }
  return 0;
}

// MatchInterPodAffinity (predicates.go:1143-1450) over the row-form counts: existing pods' required
// anti-affinity terms the pod matches (satisfiesExistingPodsAntiAffinity :1340-1379), then its own
// required affinity terms (a term no placed pod matches is waived when the pod matches it itself,
// :1405-1424) and required anti-affinity terms (:1430-1441).  Same reasons as ksim_interpod_pred.
__device__ __noinline__ uint32_t pg_interpod_pred(const KsimAff& A, const PGenArgs& g, const ksim_pod& P, int64_t i) {
  const uint32_t base = 1u << KSIM_R_POD_AFFINITY;
  const int64_t n = A.n;
  if (P.aff_ident > 0) {
    const uint64_t* mw = A.ident_anti + (int64_t)(P.aff_ident - 1) * A.carry_words;
    for (int32_t w = 0; w < A.carry_words; ++w) {
      uint64_t m = mw[w];
      while (m) {
        const int e = 64 * w + __builtin_ctzll(m);
        m &= m - 1;
        if (g.car_row[(int64_t)e * n + i] > 0) return base | (1u << KSIM_R_EXISTING_ANTI_AFFINITY);
      }
    }
  }
  if (P.aff_class <= 0) return 0;
  const int32_t* ac = A.ac + 6 * (int64_t)(P.aff_class - 1);
  for (int32_t j = ac[0], e = ac[0] + ac[1]; j < e; ++j) {
    const ksim_aff_term t = A.terms[j];
    const bool match = ksim_dom(A, t.gate_key, i) >= 0 && g.cnt_row[(int64_t)t.pair * n + i] > 0;
    if (t.kind == KSIM_AFF_REQ_AFFINITY) {
      if (!match && (!t.self_ok || g.cnt_row[(int64_t)t.exist_pair * n + i] > 0))
        return base | (1u << KSIM_R_AFFINITY_RULES);
    } else if (match) {
      return base | (1u << KSIM_R_ANTI_AFFINITY_RULES);
    }
  }
  return 0;
}

// CalculateInterPodAffinityPriority's per-node sum (interpod_affinity.go:124-214) before the
// normalisation, over the row-form counts (0 on rows without the term's key, as in Go).
__device__ __noinline__ int64_t pg_interpod_raw(const KsimAff& A, const PGenArgs& g, const ksim_pod& P, int64_t i) {
  const int64_t n = A.n;
  int64_t s = 0;
  if (P.aff_class > 0) {
    const int32_t* ac = A.ac + 6 * (int64_t)(P.aff_class - 1);
    for (int32_t j = ac[2], e = ac[2] + ac[3]; j < e; ++j) {
      const ksim_aff_term t = A.terms[j];
      s += t.weight * (int64_t)g.cnt_row[(int64_t)t.pair * n + i];
    }
  }
  if (P.aff_ident > 0) {
    const uint64_t* mw = A.ident_prio + (int64_t)(P.aff_ident - 1) * A.carry_words;
    for (int32_t w = 0; w < A.carry_words; ++w) {
      uint64_t m = mw[w];
      while (m) {
        const int e = 64 * w + __builtin_ctzll(m);
        m &= m - 1;
        s += g.car_row[(int64_t)e * n + i];
      }
    }
  }
  return s;
}

// The first failing predicate of predicatesOrdering (predicates.go:129-138) on row j (node i),
// exactly the chain of ksim_predicates_a, with the row's label / taint verdicts from the static
// word `st` and its volume mounts from LDS.  0 = fits.
__device__ __forceinline__ uint32_t pg_predicates(const KsimCtx& c, const PGenArgs& g, const PgLds& L, const ksim_pod& P,
                                                  int32_t j, int64_t i, const KsimRow& r, uint32_t st, bool aff_pod) {
  const uint32_t pr = c.preds;
  uint32_t m;
  if (pr & KSIM_P_CHECK_NODE_CONDITION) {
    m = r.fl & KSIM_COND_REASON_MASK;  // bit positions coincide with KSIM_R_*
    if (m) return m;
  }
  if ((pr & KSIM_P_CHECK_NODE_UNSCHEDULABLE) && (r.fl & KSIM_N_UNSCHEDULABLE)) return 1u << KSIM_R_UNSCHEDULABLE;
  const uint32_t sel = ((P.flags & KSIM_POD_NEED_SELECTOR) && (st & PG_ST_SEL)) ? (1u << KSIM_R_NODE_SELECTOR) : 0u;
  if (pr & KSIM_P_GENERAL) {
    m = ksim_resources(c, P, i, r) | ksim_hostname(P, i) | sel;
    if (P.port_cnt) m |= ksim_hostports(c, P, i, KsimGlobalAcc{c});
    if (m) return m;
  }
  if (pr & KSIM_P_HOSTNAME) {
    m = ksim_hostname(P, i);
    if (m) return m;
  }
  if ((pr & KSIM_P_HOST_PORTS) && P.port_cnt) {
    m = ksim_hostports(c, P, i, KsimGlobalAcc{c});
    if (m) return m;
  }
  if ((pr & KSIM_P_NODE_SELECTOR) && sel) return sel;
  if (pr & KSIM_P_RESOURCES) {
    m = ksim_resources(c, P, i, r);
    if (m) return m;
  }
  const bool vol = g.has_vol && P.vol_class > 0;
  if ((pr & KSIM_P_DISK_CONFLICT) && vol) {
    m = pg_disk_conflict(g.V, L, P.vol_class, j, i);
    if (m) return m;
  }
  if ((pr & KSIM_P_TAINTS) && (P.flags & KSIM_POD_NEED_TAINTS) && (st & PG_ST_TAINT)) return 1u << KSIM_R_TAINTS;
  if ((pr & KSIM_P_NOEXEC_TAINTS) && (P.flags & KSIM_POD_NEED_TAINTS) && (st & PG_ST_NOEXEC)) return 1u << KSIM_R_TAINTS;
  if ((pr & KSIM_P_LABEL_PRESENCE) && (r.fl & KSIM_N_LABEL_PRESENCE)) return 1u << KSIM_R_LABEL_PRESENCE;
  if ((pr & KSIM_P_SERVICE_AFFINITY) && (P.flags & KSIM_POD_NEED_SVC_AFFINITY) && (st & PG_ST_SVC))
    return 1u << KSIM_R_SERVICE_AFFINITY;
  if (vol) {
    const uint32_t which = ((pr & KSIM_P_MAX_EBS) ? KSIM_VOL_EBS : 0u) | ((pr & KSIM_P_MAX_GCE_PD) ? KSIM_VOL_GCE_PD : 0u) |
                           ((pr & KSIM_P_MAX_AZURE_DISK) ? KSIM_VOL_AZURE_DISK : 0u);
    if (which) {
      m = pg_max_volumes(g.V, L, P.vol_class, j, i, which);
      if (m) return m;
    }
    if ((pr & KSIM_P_VOLUME_ZONE) && !ksim_vol_zone_ok(g.V, P.vol_class, L.ls[j])) return 1u << KSIM_R_VOLUME_ZONE;
  }
  if ((pr & KSIM_P_MEM_PRESSURE) && (P.flags & KSIM_POD_BEST_EFFORT) && (r.fl & KSIM_N_MEM_PRESSURE))
    return 1u << KSIM_R_MEM_PRESSURE;
  if ((pr & KSIM_P_DISK_PRESSURE) && (r.fl & KSIM_N_DISK_PRESSURE)) return 1u << KSIM_R_DISK_PRESSURE;
  if ((pr & KSIM_P_INTERPOD_AFFINITY) && aff_pod) return pg_interpod_pred(g.A, g, P, i);
  return 0;
}

// Refresh row j's LDS view of its volume mounts (count, first slots, per-filter counts) from the
// HBM columns — at launch, and by the owner's wave after a commit.  One wave, lane s = slot s.
__device__ __noinline__ void pg_vol_row(const KsimVol& V, const PgLds& L, int32_t j, int64_t i, int lane) {
  const int32_t cnt = V.slot_count[i];
  uint32_t h[3] = {0, 0, 0};
  for (int32_t s0 = 0; s0 < cnt; s0 += 64) {
    const int32_t s = s0 + lane;
    uint32_t f = 0;
    if (s < cnt) {
      const uint64_t w = V.slots[(int64_t)s * V.n + i];
      if (s < L.nvs) L.vs[(int64_t)s * L.chunk + j] = w;
      f = V.key_filter[(int32_t)(w >> 32)];
    }
#pragma unroll
    for (int t = 0; t < 3; ++t) h[t] += __popcll(__ballot((f >> t) & 1u));
  }
  if (lane == 0) {
    L.vc[j] = cnt;
#pragma unroll
    for (int t = 0; t < 3; ++t) L.vh[(int64_t)t * L.chunk + j] = (uint16_t)(h[t] < 65535 ? h[t] : 65535);
  }
}

// NodeInfo.AddPod's affinity part for this workgroup's rows [lo, hi): +1 on the row-form count of
// every pair whose selector the pod's identity matches, on the rows in node w's domain of the
// pair's key; + the pod's carried amounts likewise.
__device__ __noinline__ void pg_aff_commit_rows(const KsimAff& A, const PGenArgs& g, const ksim_pod& P, int64_t w,
                                                int64_t lo, int64_t hi, int tid) {
  const int64_t n = A.n;
  if (P.aff_ident > 0) {
    const uint64_t* sm = A.ident_sel + (int64_t)(P.aff_ident - 1) * A.sel_words;
    for (int32_t c = 0; c < A.n_pair; ++c) {
      const int32_t s = A.pair_sel[c];
      if (!((sm[s >> 6] >> (s & 63)) & 1ull)) continue;
      const int32_t k = A.pair_key[c];
      const int32_t dw = ksim_dom(A, k, w);
      if (dw < 0) continue;
      if (k == 1) {  // the node pseudo key: node w's row only
        if (tid == 0 && w >= lo && w < hi) g.cnt_row[(int64_t)c * n + w] += 1;
        continue;
      }
      for (int64_t i = lo + tid; i < hi; i += PG_BS)
        if (ksim_dom(A, k, i) == dw) g.cnt_row[(int64_t)c * n + i] += 1;
    }
  }
  if (P.aff_class > 0) {
    const int32_t* ac = A.ac + 6 * (int64_t)(P.aff_class - 1);
    for (int32_t j = ac[4], e = ac[4] + ac[5]; j < e; ++j) {
      const ksim_aff_carry kc = A.carries[j];
      const int32_t k = A.carry_key[kc.term];
      const int32_t dw = ksim_dom(A, k, w);
      if (dw < 0) continue;
      for (int64_t i = lo + tid; i < hi; i += PG_BS)
        if (ksim_dom(A, k, i) == dw) g.car_row[(int64_t)kc.term * n + i] += kc.amount;
    }
  }
}

}  // namespace

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

template <int NPT>
__global__ __launch_bounds__(PG_BS) void ksim_pgen_kernel(KsimCtx c, PGenArgs g) {
  extern __shared__ __attribute__((aligned(16))) char pg_smem[];
  __shared__ int64_t s_a[4][PG_NW];                  // pass A per wave: min, max, max count, haveZones
  __shared__ unsigned long long s_z[PG_MAXZ];        // pass A zone sums of this workgroup
  __shared__ int64_t s_g[5];                         // pass A over the grid: min, max, max count, haveZones, max zone
  __shared__ int64_t s_gz[PG_MAXZ];                  // countsByZone over the grid
  __shared__ int32_t s_mx[PG_NW][KSIM_MAX_RCLASS];   // class partials per wave
  __shared__ int32_t s_cn[PG_NW][KSIM_MAX_RCLASS];
  __shared__ int32_t s_fit[PG_NW];
  __shared__ int32_t s_mode, s_blk, s_rank, s_abort;
  __shared__ uint32_t s_win;
  __shared__ int32_t s_tgt[KSIM_MAX_RCLASS];         // winning class q: its maximum (else -2)
  __shared__ int64_t s_node;
#ifdef KSIM_STAMPS
  uint64_t st_acc[8] = {};
  uint64_t t_prev = __builtin_amdgcn_s_memtime();
#endif

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int G = gridDim.x;
  const int64_t chunk = c.chunk;
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = (lo + chunk < c.n) ? lo + chunk : c.n;
  const int32_t nrows = (int32_t)(hi - lo);
  // LDS image (layout: ksim_pgen_plan)
  PgLds L;
  {
    char* q = pg_smem;
    auto take = [&](size_t b) { char* r = q; q += (b + 15) & ~(size_t)15; return r; };
    L.chunk = chunk;
    L.nvs = g.vs;
    L.ac = (int64_t*)take(chunk * 8); L.am = (int64_t*)take(chunk * 8);
    L.rc = (int64_t*)take(chunk * 8); L.rm = (int64_t*)take(chunk * 8);
    L.zc = (int64_t*)take(chunk * 8); L.zm = (int64_t*)take(chunk * 8);
    L.al = (int32_t*)take(chunk * 4); L.ct = (int32_t*)take(chunk * 4); L.fl = (uint32_t*)take(chunk * 4);
    L.ls = (int32_t*)take(chunk * 4); L.ts = (int32_t*)take(chunk * 4);
    L.sc = (int32_t*)take(chunk * 4); L.cl = (uint8_t*)take(chunk);
    L.vc = (int32_t*)take(chunk * 4); L.vh = (uint16_t*)take(chunk * 6);
    L.vs = (uint64_t*)take((size_t)g.vs * chunk * 8);
    L.st = g.st_classes ? (uint16_t*)take((size_t)g.st_classes * chunk * 2) : nullptr;
  }
  for (int32_t j = tid; j < nrows; j += PG_BS) {
    const int64_t i = lo + j;
    L.ac[j] = c.alloc_cpu[i]; L.am[j] = c.alloc_mem[i];
    L.rc[j] = c.req_cpu[i]; L.rm[j] = c.req_mem[i]; L.zc[j] = c.nz_cpu[i]; L.zm[j] = c.nz_mem[i];
    L.al[j] = c.allowed_pods[i]; L.ct[j] = c.pod_count[i]; L.fl[j] = c.flags[i];
    L.ls[j] = c.label_set[i]; L.ts[j] = c.taint_set[i];
  }
  if (g.has_vol)  // the rows' volume mounts: one wave per row
    for (int32_t j = wv; j < nrows; j += PG_NW) pg_vol_row(g.V, L, j, lo + j, lane);
  if (tid == 0) s_abort = 0;
  uint64_t counter = *c.counter;  // replicated genericScheduler.lastNodeIndex (wave 0)
  __syncthreads();
  if (L.st)  // static (pod class, row) words from the class tables
    for (int32_t k = tid; k < g.st_classes * nrows; k += PG_BS) {
      const int32_t cls = k / nrows, j = k - cls * nrows;
      L.st[(int64_t)cls * chunk + j] = (uint16_t)pg_static_word(c, cls, L.ls[j], L.ts[j]);
    }
  __syncthreads();

  for (int64_t pod = c.first; pod < c.end; ++pod) {
    const ksim_pod P = c.pods[pod];
    const int k1 = (c.w[KSIM_W_TAINT_TOLERATION] != 0) ? c.n_tt[P.cls] : 1;
    const int k2 = c.use_na ? c.n_na[P.cls] : 1;
    const int K = k1 * k2;
    const bool aff_pod = g.has_aff && (P.aff_ident > 0 || P.aff_class > 0);
    const bool ipa = aff_pod && !c.no_prio && c.w[KSIM_W_INTERPOD_AFFINITY] != 0 && ksim_interpod_prio_work(g.A, P);
    const int32_t sp = (g.has_aff && !c.no_prio && c.w[KSIM_W_SELECTOR_SPREAD] != 0) ? ksim_spread_pair(g.A, P) : -1;
    const uint32_t tag = (uint32_t)((pod - c.first + 1) & 0xFF);
    const int slot = (int)(pod % PG_NSLOT);
    // the decision's per-class map values (lane q = reduce class q), loaded off the critical path
    int64_t tv_l = 0, av_l = 0, ad_l = 0;
    if (wv == 0 && K > 1 && lane < K) {
      tv_l = c.tt_val[(int64_t)P.cls * KSIM_MAX_RCLASS + lane / k2];
      av_l = c.na_val[(int64_t)P.cls * KSIM_MAX_RCLASS + lane % k2];
      if (c.na_add) ad_l = c.na_add[(int64_t)P.cls * KSIM_MAX_RCLASS + lane % k2];
    } else if (wv == 0 && lane == 0) {
      tv_l = c.tt_val[(int64_t)P.cls * KSIM_MAX_RCLASS];
      av_l = c.na_val[(int64_t)P.cls * KSIM_MAX_RCLASS];
      if (c.na_add) ad_l = c.na_add[(int64_t)P.cls * KSIM_MAX_RCLASS];
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
      const uint32_t st = L.st ? (uint32_t)L.st[(int64_t)P.cls * chunk + j] : pg_static_word(c, P.cls, L.ls[j], L.ts[j]);
      const uint32_t m = pg_predicates(c, g, L, P, j, i, r, st, aff_pod);
      rmk[k] = m;
      if (m) continue;
      fit[k] = true;
      sc[k] = ksim_map_score(c, P, r);
      cl[k] = (k1 > 1 ? (int32_t)((st >> 4) & 15u) : 0) * k2 + (k2 > 1 ? (int32_t)((st >> 8) & 15u) : 0);
      if (ipa) raw[k] = pg_interpod_raw(g.A, g, P, i);
      if (sp >= 0) {
        cnt[k] = g.cnt_row[(int64_t)sp * c.n + i];
        zz[k] = g.A.zone_key >= 0 ? ksim_dom(g.A, g.A.zone_key, i) : -1;
      }
    }
    PG_STAMP(0);

    // ---- 2. pass A over the grid (pods that read InterPodAffinity / SelectorSpread) ----
    if (ipa || sp >= 0) {
      if (tid < PG_MAXZ) s_z[tid] = 0;
      __syncthreads();
      int64_t mn = 0, mx = 0, smx = 0, hz = 0;
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
      }
      if (ipa) { mn = wmin64(mn); mx = wmax64(mx); }
      if (sp >= 0) { smx = wmax64(smx); hz = wmax64(hz); }
      if (lane == 0) { s_a[0][wv] = mn; s_a[1][wv] = mx; s_a[2][wv] = smx; s_a[3][wv] = hz; }
      __syncthreads();
      PG_STAMP(6);
      if (wv == 0) {
        const int nz = sp >= 0 ? g.n_zone : 0;
        const int RA = 4 + nz;
        // publish this workgroup's record (lane w = word w), tagged
        if (lane < RA) {
          int64_t v;
          if (lane < 4) {
            v = s_a[lane][0];
            for (int w = 1; w < PG_NW; ++w) v = lane == 0 ? (s_a[0][w] < v ? s_a[0][w] : v) : (s_a[lane][w] > v ? s_a[lane][w] : v);
          } else {
            v = (int64_t)s_z[lane - 4];
          }
          pg_store(rec_at(g.gran, slot, lane, blockIdx.x), ((uint64_t)tag << 56) | ((uint64_t)(v + B55) & M56));
        }
        // sweep every record: lane l reads workgroups l, l + 64, ...; a batch of 8 words per poll
        int64_t a_mn = 0, a_mx = 0, a_smx = 0, a_hz = 0;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool ok = false;
        for (int w0 = 0; w0 < RA; w0 += 8) {
          uint64_t v[8][PG_MB];
          for (;;) {
            bool mine = true;
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
              for (int m = 0; m < PG_MB; ++m) {
                const int b = lane + 64 * m;
                v[u][m] = (w0 + u < RA && b < G) ? pg_load(rec_at(g.gran, slot, w0 + u, b)) : ((uint64_t)tag << 56);
                mine &= gtag(v[u][m]) == tag;
              }
            if (__all(mine)) { ok = true; break; }
            ok = false;
            if (__builtin_amdgcn_s_memrealtime() - t0 > g.spin_ticks) break;
            __builtin_amdgcn_s_sleep(1);
          }
          if (!ok) break;
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int word = w0 + u;
            if (word >= RA) break;
            int64_t acc = word == 0 ? INT64_MAX : (word < 4 ? INT64_MIN : 0);
#pragma unroll
            for (int m = 0; m < PG_MB; ++m) {
              if (lane + 64 * m >= G) continue;
              const int64_t x = (int64_t)(v[u][m] & M56) - B55;
              if (word == 0) acc = x < acc ? x : acc;
              else if (word < 4) acc = x > acc ? x : acc;
              else acc += x;
            }
            if (word == 0) a_mn = ipa ? wmin64(acc) : 0;
            else if (word == 1) a_mx = ipa ? wmax64(acc) : 0;
            else if (word == 2) a_smx = sp >= 0 ? wmax64(acc) : 0;
            else if (word == 3) a_hz = sp >= 0 ? wmax64(acc) : 0;
            else {
              const int64_t zsum = wsum64(acc);
              if (lane == 0) s_gz[word - 4] = zsum;
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
        }
      }
      __syncthreads();
      if (s_abort) break;
      const int64_t gmn = s_g[0], gmx = s_g[1], gsmx = s_g[2], ghz = s_g[3], gzm = s_g[4];
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
      }
    }
    PG_STAMP(1);

    // ---- 3. per reduce class (max, count) and fit count of this workgroup ----
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int32_t j = k * PG_BS + tid;
      if (j < nrows) { L.sc[j] = fit[k] ? (int32_t)sc[k] : -1; L.cl[j] = (uint8_t)cl[k]; }
    }
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
      int32_t n = 0;
#pragma unroll
      for (int k = 0; k < NPT; ++k) n += __popcll(__ballot(fit[k] && cl[k] == q && (int32_t)sc[k] == wm));
      if (lane == 0) { s_mx[wv][q] = wm; s_cn[wv][q] = wm < 0 ? 0 : n; }
    }
    __syncthreads();
    PG_STAMP(2);

    // ---- 4. wave 0: publish, sweep every workgroup's granules, decide ----
    if (wv == 0) {
      if (lane < K) {
        int32_t m = -1, n = 0, f = 0;
        for (int w = 0; w < PG_NW; ++w) {
          f += s_fit[w];
          if (!s_cn[w][lane]) continue;
          if (s_mx[w][lane] > m) { m = s_mx[w][lane]; n = s_cn[w][lane]; }
          else if (s_mx[w][lane] == m) n += s_cn[w][lane];
        }
        const uint64_t v = ((uint64_t)tag << 56) | (lane == 0 ? ((uint64_t)f << 44) : 0) | ((uint64_t)n << 32) |
                           (uint64_t)(uint32_t)m;
        pg_store(cls_at(g.gran, slot, lane, blockIdx.x), v);
      }
      uint64_t gv[KSIM_MAX_RCLASS][PG_MB];
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      bool ok = false;
      for (;;) {
        bool mine = true;
#pragma unroll
        for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
          if (q >= K) break;
#pragma unroll
          for (int m = 0; m < PG_MB; ++m) {
            const int b = lane + 64 * m;
            gv[q][m] = b < G ? pg_load(cls_at(g.gran, slot, q, b)) : ((uint64_t)tag << 56);
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
      int mode = 0, blk = -1, rank = 0;
      uint32_t win = 0;
      int32_t tgt_l = -2;  // lane q: class q's maximum if q wins
      if (!ok) {
        mode = -1;
        if (lane == 0) atomicOr(c.err, 4);
      } else {
        int32_t f = 0;
#pragma unroll
        for (int m = 0; m < PG_MB; ++m) f += (lane + 64 * m < G) ? gfit(gv[0][m]) : 0;
        const int32_t F = ksimw::sum_i32(f);
        int32_t mq_l = -1, cq_l = 0;  // lane q: class q's global maximum and its count
#pragma unroll
        for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
          if (q >= K) break;
          int32_t mm = -1, nn = 0;
#pragma unroll
          for (int m = 0; m < PG_MB; ++m) {
            if (lane + 64 * m >= G) continue;
            const int32_t cn = gcnt(gv[q][m]), s = gscore(gv[q][m]);
            if (!cn) continue;
            if (s > mm) { mm = s; nn = cn; }
            else if (s == mm) nn += cn;
          }
          const int32_t Mq = ksimw::max_i32(nn ? mm : -1);
          const int32_t Cq = ksimw::sum_i32((nn && mm == Mq) ? nn : 0);
          mq_l = lane == q ? Mq : mq_l;
          cq_l = lane == q ? Cq : cq_l;
        }
        if (F > 0) {
          mode = 1;
          int64_t ix = 0;
          if (F > 1) {  // generic_scheduler.go:153-156: a single fit skips selectHost
            mode = 2;
            // lane q = reduce class q: NormalizeReduce over the filtered set, weighted totals
            // (reduce.go:29-64, generic_scheduler.go:632-639), the best total and its classes
            const bool live = lane < K && cq_l != 0;
            int64_t mxT = 0, mxA = 0;
            if (k1 > 1 || c.w[KSIM_W_TAINT_TOLERATION]) mxT = wmax64(live ? tv_l : 0);
            if (k2 > 1 || c.w[KSIM_W_NODE_AFFINITY]) mxA = wmax64(live ? av_l : 0);
            uint64_t t = (uint64_t)(int64_t)mq_l + (uint64_t)ad_l;
            if (c.w[KSIM_W_TAINT_TOLERATION]) t += (uint64_t)c.w[KSIM_W_TAINT_TOLERATION] * (uint64_t)ksim_norm(tv_l, mxT, true);
            if (c.w[KSIM_W_NODE_AFFINITY]) t += (uint64_t)c.w[KSIM_W_NODE_AFFINITY] * (uint64_t)ksim_norm(av_l, mxA, false);
            const int64_t tot = live ? (int64_t)t : INT64_MIN;
            const int64_t best = wmax64(tot);
            const uint64_t wbm = __ballot(live && tot == best);
            win = (uint32_t)wbm;
            const int32_t C = ksimw::sum_i32(((wbm >> lane) & 1ull) ? cq_l : 0);
            tgt_l = ((wbm >> lane) & 1ull) ? mq_l : -2;
            ix = (counter >> 32) ? (int64_t)(counter % (uint64_t)C) : (int64_t)((uint32_t)counter % (uint32_t)C);
            counter += 1;  // generic_scheduler.go:192-195
          }
          // locate the workgroup holding the ix-th match from the top (lane-major workgroup order:
          // lane l holds l, l + 64, ...; name rank grows with the workgroup index)
          int32_t bm[PG_MB];
#pragma unroll
          for (int m = 0; m < PG_MB; ++m) {
            const int b = lane + 64 * m;
            int32_t s = 0;
            if (b < G) {
              if (mode == 1) {
                s = gfit(gv[0][m]);
              } else {
#pragma unroll
                for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
                  if (q >= K) break;
                  if (!((win >> q) & 1u)) continue;
                  const int32_t Mq = __builtin_amdgcn_readlane(mq_l, q);
                  if (gcnt(gv[q][m]) && gscore(gv[q][m]) == Mq) s += gcnt(gv[q][m]);
                }
              }
            }
            bm[m] = s;
          }
          // matches in workgroups above b = (lanes above, same m) + (every lane, higher m)
          int64_t above = 0;
          int found = -1, rk = 0;
          for (int m = PG_MB - 1; m >= 0 && found < 0; --m) {
            if (64 * m >= G) continue;
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
          if (found < 0) { mode = -1; if (lane == 0) atomicOr(c.err, 2); }
          blk = found;
          rank = rk;
        }
      }
      if (lane < KSIM_MAX_RCLASS) s_tgt[lane] = tgt_l;
      if (lane == 0) { s_mode = mode; s_blk = blk; s_rank = rank; s_win = win; s_node = -1; }
    }
    __syncthreads();
    PG_STAMP(3);
    const int mode = s_mode;
    if (mode < 0) break;  // uniform: every workgroup reached the same verdict

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

    // ---- 6. the owner picks the row (the rank-th match from the top) and commits it ----
    const bool owner = s_blk == (int)blockIdx.x;
    // pods whose affinity counts change shared topology domains (zones, "anywhere"): every
    // workgroup applies them, so the owner publishes the node (commit word, tagged) and the others
    // wait for it; otherwise only the owner's rows change (node keys, injective label keys)
    const bool shared = aff_pod && !c.no_commit &&
                        ((P.aff_ident > 0 && g.ident_shared[P.aff_ident - 1]) ||
                         (P.aff_class > 0 && g.aclass_shared[P.aff_class - 1]));
    if (owner && wv == 0) {
      const uint32_t win = s_win;
      int32_t rr = s_rank, jsel = -1;
      const int nseg = (nrows + 63) / 64;
      for (int s0 = nseg - 1; s0 >= 0 && jsel < 0; --s0) {
        const int32_t j = s0 * 64 + lane;
        bool mt = false;
        if (j < nrows) {
          const int32_t e = L.sc[j];
          if (mode == 1) mt = e >= 0;
          else mt = e >= 0 && ((win >> L.cl[j]) & 1u) && e == s_tgt[L.cl[j]];
        }
        const uint64_t bl = __ballot(mt);
        const int nb = __popcll(bl);
        if (rr >= nb) { rr -= nb; continue; }
        const bool is = ((bl >> lane) & 1ull) && __popcll((bl >> lane) >> 1) == rr;
        jsel = s0 * 64 + (__builtin_ffsll((long long)__ballot(is)) - 1);
      }
      if (jsel < 0) {
        if (lane == 0) { atomicOr(c.err, 2); s_abort = 1; }
      } else {
        const int64_t w = lo + jsel;
        if (lane == 0) {
          s_node = w;
          c.out_node[pod] = (int32_t)w;
          if (shared) pg_store(g.gran + PG_COMMIT_OFF + slot, ((uint64_t)tag << 56) | (uint64_t)w);
          if (!c.no_commit) {
            // NodeInfo.AddPod on the row (node_info.go:318-341): LDS columns, then HBM side columns
            L.rc[jsel] += P.add_cpu; L.rm[jsel] += P.add_mem; L.zc[jsel] += P.nz_cpu; L.zm[jsel] += P.nz_mem;
            L.ct[jsel] += 1;
            if (P.add_gpu | P.add_eph) {
              const int64_t gg = c.req_gpu[w] + P.add_gpu, ge = c.req_eph[w] + P.add_eph;
              c.req_gpu[w] = gg;
              c.req_eph[w] = ge;
              uint32_t fl = L.fl[jsel] & ~(KSIM_N_GPU_OVER | KSIM_N_EPH_OVER);
              if (c.alloc_gpu[w] < gg) fl |= KSIM_N_GPU_OVER;
              if (c.alloc_eph[w] < ge) fl |= KSIM_N_EPH_OVER;
              L.fl[jsel] = fl;
            }
            for (int32_t s = 0; s < P.scalar_cnt; ++s) {
              const ksim_scalar_req q = c.pod_scalars[P.scalar_off + s];
              c.req_scalar[(int64_t)q.col * c.n + w] += q.add;
            }
            for (int32_t k = 0; k < P.port_cnt; ++k) {  // HostPortInfo.Add (utils.go:45-60)
              const uint64_t key = c.pod_ports[P.port_off + k];
              const int32_t cnt0 = c.port_count[w];
              bool dup = false;
              for (int32_t s = 0; s < cnt0; ++s)
                if (c.ports[(int64_t)s * c.n + w] == key) { dup = true; break; }
              if (dup) continue;
              if (cnt0 >= c.port_slots) { atomicOr(c.err, 1); continue; }
              c.ports[(int64_t)cnt0 * c.n + w] = key;
              c.port_count[w] = cnt0 + 1;
            }
            if (g.has_vol && P.vol_class > 0) ksim_vol_commit(g.V, P, w, 1, c.err);
          }
        }
        if (!c.no_commit && g.has_vol && P.vol_class > 0) {
          // the row's LDS view of its mounts follows the HBM columns lane 0 just wrote
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          pg_vol_row(g.V, L, jsel, w, lane);
        }
      }
    } else if (shared && tid == 0) {
      // the chosen node, from the owner's commit word
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint64_t v;
      while (gtag(v = pg_load(g.gran + PG_COMMIT_OFF + slot)) != tag) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > g.spin_ticks) { atomicOr(c.err, 4); s_abort = 1; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      s_node = (int64_t)(v & M56);
    }
    __syncthreads();
    PG_STAMP(4);
    if (s_abort) break;
    // ---- 7. the pod's affinity counts on this workgroup's rows (NodeInfo.AddPod's affinity part) ----
    if (aff_pod && !c.no_commit && (shared || owner)) {
      pg_aff_commit_rows(g.A, g, P, s_node, lo, hi, tid);
      __syncthreads();
    }
    PG_STAMP(5);
  }
  // the table is authoritative in HBM between calls: write the owned rows back
  __syncthreads();
  for (int32_t j = tid; j < nrows; j += PG_BS) {
    const int64_t i = lo + j;
    c.req_cpu[i] = L.rc[j]; c.req_mem[i] = L.rm[j]; c.nz_cpu[i] = L.zc[j]; c.nz_mem[i] = L.zm[j];
    c.pod_count[i] = L.ct[j]; c.flags[i] = L.fl[j];
  }
  if (blockIdx.x == 0 && tid == 0) {
    *c.counter = counter;
    *c.cursor = c.end;
#ifdef KSIM_STAMPS
    for (int k = 0; k < 8; ++k) c.dbg[k] += st_acc[k];
#endif
  }
}

// Canonical per-domain counts (ksim_load_affinity's cnt / carried, read by the launch kernels and
// the per-pod entry points) <-> the row form (to_rows = 1: build; 0: fold back — every row of a
// domain holds the same value, so concurrent identical stores are benign).
__global__ void ksim_pgen_rows_kernel(const KsimAff* __restrict__ Ap, int32_t* cnt_row, int64_t* car_row, int32_t n_pair,
                                      int32_t n_carry, int32_t to_rows) {
  const KsimAff& A = *Ap;
  const int64_t n = A.n;
  const int64_t total = (int64_t)(n_pair + n_carry) * n;
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = x / n, i = x - c * n;
    if (c < n_pair) {
      const int32_t d = ksim_dom(A, A.pair_key[c], i);
      if (to_rows) cnt_row[x] = d >= 0 ? A.cnt[A.pair_off[c] + d] : 0;
      else if (d >= 0) A.cnt[A.pair_off[c] + d] = cnt_row[x];
    } else {
      const int64_t e = c - n_pair;
      const int32_t d = ksim_dom(A, A.carry_key[e], i);
      if (to_rows) car_row[e * n + i] = d >= 0 ? A.carried[A.carry_off[e] + d] : 0;
      else if (d >= 0) A.carried[A.carry_off[e] + d] = car_row[e * n + i];
    }
  }
}

extern "C" hipError_t ksim_pgen_rows(const KsimAff* aff_dev, int32_t* cnt_row, int64_t* car_row, int32_t n_pair,
                                     int32_t n_carry, int64_t n, int to_rows, hipStream_t s) {
  const int64_t total = (int64_t)(n_pair + n_carry) * n;
  if (total <= 0) return hipSuccess;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(ksim_pgen_rows_kernel, dim3(grid), dim3(256), 0, s, aff_dev, cnt_row, car_row, n_pair, n_carry,
                     to_rows);
  return hipGetLastError();
}

extern "C" size_t ksim_pgen_gran_bytes(void) { return (size_t)PG_GRAN_WORDS * sizeof(uint64_t); }
extern "C" int ksim_pgen_max_zones(void) { return PG_MAXZ; }

// Grid and rows per workgroup: up to 256 rows per workgroup at one row per thread (more
// workgroups only widen the exchange), up to 4 rows per thread once the grid reaches 256.
extern "C" int ksim_pgen_config(int64_t n, int max_grid, int* grid, int* npt) {
  if (n <= 0) return 0;
  int cap = PG_MAXG;
  if (max_grid > 0 && max_grid < cap) cap = max_grid;
  for (int k : {1, 2, 4}) {
    const int64_t g = (n + (int64_t)PG_BS * k - 1) / ((int64_t)PG_BS * k);
    if (g <= cap) {
      *grid = (int)g;
      *npt = k;
      return 1;
    }
  }
  return 0;
}

// Dynamic LDS of the kernel for `chunk` rows: the fixed per-row arrays, then as many volume slots
// per row (<= PG_VS_MAX, <= the table's) and the static (class, row) words when they fit.
extern "C" size_t ksim_pgen_plan(int64_t chunk, int32_t n_classes, int32_t vol_slots, int32_t* vs, int32_t* st_classes) {
  auto al = [](size_t b) { return (b + 15) & ~(size_t)15; };
  const size_t C = (size_t)chunk;
  size_t base = 6 * al(C * 8) + 5 * al(C * 4) + al(C * 4) + al(C) + al(C * 4) + al(C * 6);
  const size_t st = al((size_t)n_classes * C * 2);
  *st_classes = (base + st <= (size_t)PG_LDS_BUDGET) ? n_classes : 0;
  if (*st_classes) base += st;
  int32_t v = std::min<int32_t>(vol_slots, PG_VS_MAX);
  while (v > 0 && base + al((size_t)v * C * 8) > (size_t)PG_LDS_BUDGET) --v;
  *vs = v > 0 ? v : 0;
  return base + al((size_t)(*vs) * C * 8) + 16;
}

template <int NPT>
static hipError_t launch_pgen(const KsimCtx* c, const PGenArgs* g, int grid, size_t lds, hipStream_t s) {
  hipError_t e = ksim_check_coresident(ksim_pgen_kernel<NPT>, grid, PG_BS, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((ksim_pgen_kernel<NPT>), dim3(grid), dim3(PG_BS), lds, s, *c, *g);
  return hipGetLastError();
}

extern "C" hipError_t ksim_launch_pgen(const KsimCtx* c, const PGenArgs* g, int grid, int npt, hipStream_t s) {
  int32_t vs = 0, stc = 0;
  const size_t lds = ksim_pgen_plan(c->chunk, c->n_classes_dev, g->has_vol ? g->V.vol_slots : 0, &vs, &stc);
  if (vs != g->vs || stc != g->st_classes) return hipErrorInvalidValue;  // the caller plans with ksim_pgen_plan
  switch (npt) {
    case 1: return launch_pgen<1>(c, g, grid, lds, s);
    case 2: return launch_pgen<2>(c, g, grid, lds, s);
    default: return launch_pgen<4>(c, g, grid, lds, s);
  }
}
