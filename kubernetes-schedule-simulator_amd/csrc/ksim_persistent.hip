// ksim_persistent.hip — persistent-kernel mode (KSIM_MODE_PERSISTENT).
//
// One launch walks the whole pod queue.  Workgroup b owns the contiguous name-rank range
// [b*chunk, (b+1)*chunk) of the node table and keeps those rows in LDS for the whole launch
// (only the owner of a node reads or writes it, so node state needs no cross-workgroup
// coherence).  Each 512-thread workgroup splits into one CONTROL wave and seven ROW waves:
//
//   control wave (wave 0)                      row waves (1..7)
//   a. publish the partial of pod p            b. evaluate pod p+1 against the rows,
//      (tagged 8-byte granules)                   speculatively (as if p's winner were not
//   c. sweep every workgroup's granules of p,     in this range — true for all workgroups
//      decide (findNodesThatFit →                 but one); wave-level (max, count) into LDS
//      PrioritizeNodes → selectHost,
//      core/generic_scheduler.go:112-198)
//   ------------------------------- barrier -------------------------------
//   d. owner of p's winner only: pick the exact node from the p scores in registers, commit
//      it into LDS (NodeInfo.AddPod), re-evaluate that one row for p+1 and redo its wave's
//      partial.  Then the control wave combines the row waves' partials of p+1.
//
// so the full-table evaluation of the next pod runs concurrently with the exchange, and the
// critical path per pod is publish → sweep → decide → (owner) one-row fix-up.
// lastNodeIndex is replicated in every workgroup's control wave.  Granules are
// double-buffered by pod parity with an 8-bit pod tag: a workgroup that publishes pod p has
// seen every workgroup's pod p-1 partial, so nobody still reads the p-2 slot it overwrites.
// Every spin is bounded (2 s) and reports through the error word.  Pod descriptors stream
// through a 4-slot LDS ring two pods ahead, so no 128-byte descriptor is pinned in SGPRs.
//
// Granule q of a workgroup: tag:8 | fit:12 (q = 0 only) | count:12 | score:32 (class q max,
// -1 = no fit node of that class).  Scores < 2^31 and chunks <= 4095 rows (host checks).
// Sweep lane l reads workgroups [l*MAXB, l*MAXB+MAXB): name-rank order is lane-major, so the
// matches above a workgroup are one DPP prefix sum away.
#include "ksim_fast.h"
#include "ksim_wave.h"

namespace {

constexpr int GR = KSIM_MAX_RCLASS;                  // granules per workgroup per slot
constexpr int MAXB = 4;                              // workgroups per sweep lane (grid <= 256)
constexpr int RING = 16;                             // pod-descriptor ring slots in LDS
constexpr int RING_FILL = 8;                         // descriptors fetched per refill
constexpr uint64_t SPIN_LIMIT_TICKS = 200000000ull;  // s_memrealtime ticks at 100 MHz = 2 s
constexpr int NSLOT = 4;                             // granule slots (pod mod NSLOT)
constexpr int MAXG = 64 * MAXB;                      // workgroups a slot is sized for
constexpr int KF = 4;                                // reduce classes polled per round trip

typedef __attribute__((address_space(1))) uint64_t gu64;

__device__ __forceinline__ void store_granule(uint64_t* g, uint64_t v) {
  __hip_atomic_store((gu64*)g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t load_granule(const uint64_t* g) {
  return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// speculative partial of workgroup b for the pod in `slot`, and the previous owner's correction
// Dense layout [slot][q][pos(b)]: one poll of class 0 touches 2 KiB (16 lines) instead of a
// line per workgroup.  pos(b) = (b % MAXB) * 64 + b / MAXB, so the sweep's j-th load of lane l
// (position j * 64 + l, coalesced across the wave) is workgroup l * MAXB + j.
__device__ __forceinline__ uint64_t* spec_at(uint64_t* gr, int slot, int b, int q) {
  return gr + ((int64_t)slot * GR + q) * MAXG + (b % MAXB) * 64 + b / MAXB;
}
__device__ __forceinline__ uint64_t* fix_at(uint64_t* gr, int slot, int q) {
  return gr + (int64_t)NSLOT * MAXG * GR + (int64_t)slot * GR + q;
}
__device__ __forceinline__ uint64_t* gran_at(uint64_t* gr, int slot, int b, int q, int X) {
  return b == X ? fix_at(gr, slot, q) : spec_at(gr, slot, b, q);
}
__device__ __forceinline__ uint32_t gtag(uint64_t v) { return (uint32_t)(v >> 56); }
__device__ __forceinline__ int32_t gfit(uint64_t v) { return (int32_t)((v >> 44) & 0xFFF); }
__device__ __forceinline__ int32_t gcnt(uint64_t v) { return (int32_t)((v >> 32) & 0xFFF); }
__device__ __forceinline__ int32_t gscore(uint64_t v) { return (int32_t)(uint32_t)v; }

#ifdef KSIM_STAMPS
// phase cycle sums kept in registers of block 0's control wave, written once at the end
#define STAMP(k)                                         \
  do {                                                   \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();   \
    st_acc[k] += t_ - t_prev;                           \
    t_prev = t_;                                        \
  } while (0)
// owner-side phase durations, summed over whichever workgroup owns each pod
#define OSTAMP(k)                                                        \
  do {                                                                   \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                   \
    if (lane == 0) atomicAdd((unsigned long long*)&c.dbg[k], t_ - o_prev); \
    o_prev = t_;                                                         \
  } while (0)
#else
#define OSTAMP(k) \
  do {            \
  } while (0)
#define STAMP(k) \
  do {           \
  } while (0)
#endif

// Packed evaluation of one row for one pod: -1 = does not fit, else class:4 | score:27
// (map scores < 2^27, host-checked; reduce classes < 16).
constexpr int EV_SHIFT = 27;
__device__ __forceinline__ int32_t ev_pack(bool fit, int32_t cl, int32_t sc) { return fit ? (cl << EV_SHIFT) | sc : -1; }
__device__ __forceinline__ int32_t ev_cls(int32_t e) { return e >> EV_SHIFT; }
__device__ __forceinline__ int32_t ev_score(int32_t e) { return e & ((1 << EV_SHIFT) - 1); }

struct Rows {  // LDS image of the owned rows (SoA)
  int64_t *ac, *am, *rc, *rm, *zc, *zm;
  double *dac, *dam;  // alloc as float64 (derived, for the fast path)
  int32_t *allowed, *count;
  uint32_t* fl;
  int32_t* ev;  // [2][rows] per pod parity: packed evaluation of the row (ev_pack)
  int32_t *ls, *ts;  // label-set / taint-set id of the row
};

// 6 x i64 + 2 x f64 + 3 x i32 + 2 x i32 evaluations + 2 x i32 set ids, padded
constexpr int LDS_ROW_BYTES = 8 * 8 + 3 * 4 + 2 * 4 + 2 * 4 + 4;  // 96

extern __shared__ __attribute__((aligned(16))) char ksim_smem[];  // dynamic LDS: the row image

__device__ __forceinline__ Rows carve(char* smem, int rows) {
  Rows r;
  int64_t* p = reinterpret_cast<int64_t*>(smem);
  r.ac = p; r.am = p + rows; r.rc = p + 2 * rows; r.rm = p + 3 * rows; r.zc = p + 4 * rows; r.zm = p + 5 * rows;
  double* d = reinterpret_cast<double*>(p + 6 * rows);
  r.dac = d; r.dam = d + rows;
  int32_t* q = reinterpret_cast<int32_t*>(d + 2 * rows);
  r.allowed = q; r.count = q + rows;
  r.fl = reinterpret_cast<uint32_t*>(q + 2 * rows);
  r.ev = q + 3 * rows;
  r.ls = q + 5 * rows;
  r.ts = q + 6 * rows;
  return r;
}

}  // namespace

// Dynamic-LDS plan of a workgroup beyond the rows (host-computed in ksim_launch_persistent):
// the rows' host ports and the pod-class tables are staged too when they fit, so the row waves
// — the CU that polls the exchange — issue no global loads while evaluating (a loaded consumer
// CU pays 2.5-2.9 us per hand-off instead of 1.1, MI355X_MICROARCH.md handoff-1to1).
struct PLayout {
  int32_t ps;          // port slots staged per row (0: ports read from HBM)
  int32_t tables;      // 1: sel_ok / taint_ok / noexec_ok / tt_class / na_class staged
  int32_t off_pc, off_pk, off_sel, off_tok, off_nok, off_ttc, off_nac;  // byte offsets in ksim_smem
  int32_t off_ttv, off_nav;  // [C][KSIM_MAX_RCLASS] reduce-class map values (int64)
};

namespace {

// The general evaluation's reads beyond the row, from LDS (KsimGlobalAcc's LDS twin).
struct LdsAcc {
  const KsimCtx& c;
  const PLayout& L;
  int64_t lo;
  int rows;
  const int32_t* ls;
  const int32_t* ts;
  __device__ __forceinline__ const uint32_t* sel() const {
    return L.tables ? reinterpret_cast<const uint32_t*>(ksim_smem + L.off_sel) : c.sel_ok;
  }
  __device__ __forceinline__ bool sel_ok(const ksim_pod& P, int64_t i) const {
    return ksim_bit(sel(), P.cls, c.lwords, ls[i - lo]);
  }
  __device__ __forceinline__ bool taint_ok(const ksim_pod& P, int64_t i) const {
    const uint32_t* t = L.tables ? reinterpret_cast<const uint32_t*>(ksim_smem + L.off_tok) : c.taint_ok;
    return ksim_bit(t, P.cls, c.twords, ts[i - lo]);
  }
  __device__ __forceinline__ bool noexec_ok(const ksim_pod& P, int64_t i) const {
    const uint32_t* t = L.tables ? reinterpret_cast<const uint32_t*>(ksim_smem + L.off_nok) : c.noexec_ok;
    return ksim_bit(t, P.cls, c.twords, ts[i - lo]);
  }
  __device__ __forceinline__ bool port_conflict(int64_t i, uint64_t want) const {
    if (!L.ps) return ksim_port_conflict(c, i, want);
    const int j = (int)(i - lo);
    const int32_t cnt = reinterpret_cast<const int32_t*>(ksim_smem + L.off_pc)[j];
    const uint64_t* pk = reinterpret_cast<const uint64_t*>(ksim_smem + L.off_pk);
    const uint32_t wip = (uint32_t)(want >> 40);
    const uint64_t wpp = want & 0xFFFFFFFFFFull;  // HostPortInfo.CheckConflict (utils.go:101-130)
    for (int32_t s = 0; s < cnt; ++s) {
      const uint64_t e = pk[s * rows + j];
      if ((e & 0xFFFFFFFFFFull) != wpp) continue;
      const uint32_t eip = (uint32_t)(e >> 40);
      if (wip == 0 || eip == 0 || eip == wip) return true;
    }
    return false;
  }
  __device__ __forceinline__ int tt_class(const ksim_pod& P, int64_t i) const {
    const uint8_t* t = L.tables ? reinterpret_cast<const uint8_t*>(ksim_smem + L.off_ttc) : c.tt_class;
    return t[(int64_t)P.cls * c.n_taint_sets + ts[i - lo]];
  }
  __device__ __forceinline__ int na_class(const ksim_pod& P, int64_t i) const {
    const uint8_t* t = L.tables ? reinterpret_cast<const uint8_t*>(ksim_smem + L.off_nac) : c.na_class;
    return t[(int64_t)P.cls * c.n_label_sets + ls[i - lo]];
  }
};

// Commit of the columns that stay in HBM (gpu, ephemeral, scalars, ports) and of the
// over-commit bits (node_info.go:318-341, utils.go:45-60).  Single thread of the owner.
__device__ __noinline__ uint32_t commit_side(const KsimCtx* __restrict__ cg, const ksim_pod* Pp, int64_t w, uint32_t fl,
                                             int32_t ports) {
  const KsimCtx& c = *cg;
  const ksim_pod& P = *Pp;
  const int64_t g = c.req_gpu[w] + P.add_gpu;
  const int64_t e = c.req_eph[w] + P.add_eph;
  c.req_gpu[w] = g;
  c.req_eph[w] = e;
  fl &= ~(KSIM_N_GPU_OVER | KSIM_N_EPH_OVER);
  if (c.alloc_gpu[w] < g) fl |= KSIM_N_GPU_OVER;
  if (c.alloc_eph[w] < e) fl |= KSIM_N_EPH_OVER;
  for (int32_t s = 0; s < P.scalar_cnt; ++s) {
    const ksim_scalar_req q = c.pod_scalars[P.scalar_off + s];
    c.req_scalar[(int64_t)q.col * c.n + w] += q.add;
  }
  for (int32_t k = 0; ports && k < P.port_cnt; ++k) {
    const uint64_t key = c.pod_ports[P.port_off + k];
    const int32_t cnt = c.port_count[w];
    bool dup = false;
    for (int32_t s = 0; s < cnt; ++s)
      if (c.ports[(int64_t)s * c.n + w] == key) { dup = true; break; }
    if (dup) continue;
    if (cnt >= c.port_slots) { atomicOr(c.err, 1); continue; }
    c.ports[(int64_t)cnt * c.n + w] = key;
    c.port_count[w] = cnt + 1;
  }
  return fl;
}

// HostPortInfo.Add of the pod's ports on row j when the rows' ports are staged in LDS: the set
// is read from LDS, new keys written to LDS and HBM (stores only, nothing waits on HBM).
__device__ __noinline__ void commit_ports_lds(const KsimCtx* __restrict__ cg, const ksim_pod* Pp, int64_t w, int32_t j,
                                              int32_t rows, int32_t off_pc, int32_t off_pk) {
  const KsimCtx& c = *cg;
  const ksim_pod& P = *Pp;
  int32_t* pc = reinterpret_cast<int32_t*>(ksim_smem + off_pc);
  uint64_t* pk = reinterpret_cast<uint64_t*>(ksim_smem + off_pk);
  int32_t cnt = pc[j];
  for (int32_t k = 0; k < P.port_cnt; ++k) {
    const uint64_t key = c.pod_ports[P.port_off + k];
    bool dup = false;
    for (int32_t s = 0; s < cnt; ++s)
      if (pk[s * rows + j] == key) { dup = true; break; }
    if (dup) continue;
    if (cnt >= c.port_slots) { atomicOr(c.err, 1); continue; }
    pk[cnt * rows + j] = key;
    c.ports[(int64_t)cnt * c.n + w] = key;
    cnt += 1;
  }
  pc[j] = cnt;
  c.port_count[w] = cnt;
}

// Total score of reduce class q once the per-class maxima over the filtered set are known
// (NormalizeReduce, priorities/reduce.go:29-64; weighted sum generic_scheduler.go:632-639).
// tv / av: the class's TaintToleration / NodeAffinity map values (prefetched per pod).
__device__ __forceinline__ int64_t class_total(const KsimCtx& c, int64_t tv, int64_t av, int64_t base, int64_t mxT,
                                               int64_t mxA) {
  uint64_t t = (uint64_t)base;
  if (c.w[KSIM_W_TAINT_TOLERATION]) t += (uint64_t)c.w[KSIM_W_TAINT_TOLERATION] * (uint64_t)ksim_norm(tv, mxT, true);
  if (c.w[KSIM_W_NODE_AFFINITY]) t += (uint64_t)c.w[KSIM_W_NODE_AFFINITY] * (uint64_t)ksim_norm(av, mxA, false);
  return (int64_t)t;
}

// wave-wide maximum of a 64-bit value: the DPP int32 reduction when every lane's value fits
// (the common case: counts, weights, scores), else a shuffle tree (ds_bpermute, ~10x slower)
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
  if (__all(v >= INT32_MIN && v <= INT32_MAX)) return ksimw::max_i32((int32_t)v);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t t = __shfl_xor(v, o, 64);
    v = t > v ? t : v;
  }
  return v;
}

// 64-bit value of lane q (wave-uniform q)
__device__ __forceinline__ int64_t readlane64(int64_t v, int q) {
  return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)((uint64_t)v >> 32), q) << 32) |
                   (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)v, q));
}

// General per-row evaluation (any supported pod), everything it reads in LDS (LdsAcc) except
// the gpu / ephemeral / scalar columns of pods requesting them.  Reads the context through a
// pointer to its device-memory copy, so no kernel-argument copy goes to scratch.
struct RowEval {
  int32_t sc;
  uint32_t rm;
  int32_t cl;
  int32_t fit;
};

typedef __attribute__((address_space(3))) const KsimCtx lds_ctx;
typedef __attribute__((address_space(3))) const PLayout lds_layout;
typedef __attribute__((address_space(3))) const ksim_pod lds_pod;

// One out-of-line copy shared by the row waves, the owner's pre-evaluation and its fix-up: its
// context, layout and pod are LDS copies, so nothing it reads for a plain pod leaves the CU.
__device__ __noinline__ RowEval eval_row_general(lds_ctx* cl, lds_layout* Ll, lds_pod* Pl, int chunk, int64_t i,
                                                 int64_t j) {
  const KsimCtx& c = *(const KsimCtx*)cl;
  const PLayout& Lp = *(const PLayout*)Ll;
  const ksim_pod& P = *(const ksim_pod*)Pl;
  const int k1 = P.reserved[0], k2 = P.reserved[1];
  const Rows R = carve(ksim_smem, chunk);
  const LdsAcc acc{c, Lp, i - j, chunk, R.ls, R.ts};
  KsimRow r;
  r.ac = R.ac[j]; r.am = R.am[j]; r.rc = R.rc[j]; r.rm = R.rm[j]; r.zc = R.zc[j]; r.zm = R.zm[j];
  r.allowed = R.allowed[j]; r.count = R.count[j]; r.fl = R.fl[j];
  const uint32_t m = ksim_predicates_a(c, P, i, r, acc);
  RowEval e;
  e.fit = (m == 0);
  e.rm = m;
  // ksim_map_score through ksim_fast.h's float64 form (bit-identical; out-of-line beyond 2^49)
  e.sc = c.no_prio ? 0
                   : (int32_t)ksim_fast_score(P.nz_cpu + r.zc, r.ac, R.dac[j], P.nz_mem + r.zm, r.am, R.dam[j],
                                              c.w[KSIM_W_LEAST_REQUESTED], c.w[KSIM_W_MOST_REQUESTED], c.w[KSIM_W_BALANCED]);
  e.cl = (k1 * k2 > 1) ? ksim_rclass_a(P, i, k1, k2, acc) : 0;
  return e;
}

}  // namespace

template <int BS, int NPT>
__global__ __launch_bounds__(BS) void ksim_persistent_kernel(KsimCtx c, const KsimCtx* __restrict__ cg,
                                                             uint64_t* granules, PLayout L) {
  constexpr int NW = BS / 64;
  constexpr int RT = BS - 64;  // row threads
  __shared__ int32_t s_mx[2][NW][KSIM_MAX_RCLASS];   // per row wave, double-buffered by pod parity
  __shared__ int32_t s_cnt[2][NW][KSIM_MAX_RCLASS];
  __shared__ int32_t s_fit[2][NW];
  __shared__ uint64_t s_fm[2][NPT][NW];  // single-class pods: per 64-row segment, fit rows
  __shared__ uint64_t s_bm[2][NPT][NW];  // ... and rows at the wave maximum
  __shared__ int32_t s_fix[2][2];  // per pod parity: {row the owner re-evaluated (-1 none), its reason mask}
  __shared__ int32_t s_hist[KSIM_NREASONS];
  __shared__ int32_t s_M[KSIM_MAX_RCLASS];
  __shared__ uint64_t s_gq[KSIM_MAX_RCLASS - 1][MAXG];  // control wave: granules of classes >= 1 (by b)
  __shared__ int32_t s_C[KSIM_MAX_RCLASS];
  __shared__ int32_t s_mode;
  __shared__ int32_t s_arr;  // row-wave arrivals (the last one of a pod publishes)
  __shared__ __attribute__((aligned(16))) ksim_pod s_pod[RING];
  __shared__ PLayout s_L;
  __shared__ KsimCtx s_ctx;  // the evaluation's copy of the context (LDS reads, no K$ misses)
#ifdef KSIM_STAMPS
  uint64_t st_acc[16] = {};
#endif

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int rt = tid - 64;  // row-thread index (row waves only)
  const int G = gridDim.x;
  const int64_t chunk = c.chunk;
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = (lo + chunk < c.n) ? lo + chunk : c.n;
  const int32_t nrows = (int32_t)(hi - lo);
  Rows R = carve(ksim_smem, (int)chunk);
  const uint32_t preds = c.preds;
  const int64_t wl = c.w[KSIM_W_LEAST_REQUESTED], wmr = c.w[KSIM_W_MOST_REQUESTED], wb = c.w[KSIM_W_BALANCED];
  const bool no_prio = c.no_prio != 0;

  for (int32_t j = tid; j < nrows; j += BS) {  // stage the owned rows into LDS
    const int64_t i = lo + j;
    const int64_t ac = c.alloc_cpu[i], am = c.alloc_mem[i];
    R.ac[j] = ac; R.am[j] = am;
    R.dac[j] = (double)ac;
    R.dam[j] = (double)am;
    R.rc[j] = c.req_cpu[i]; R.rm[j] = c.req_mem[i];
    R.zc[j] = c.nz_cpu[i]; R.zm[j] = c.nz_mem[i];
    R.allowed[j] = c.allowed_pods[i]; R.count[j] = c.pod_count[i]; R.fl[j] = c.flags[i];
    R.ls[j] = c.label_set[i]; R.ts[j] = c.taint_set[i];
    if (L.ps) {  // the rows' host ports (HostPortInfo), slot-major like the HBM column
      reinterpret_cast<int32_t*>(ksim_smem + L.off_pc)[j] = c.port_count[i];
      for (int32_t q = 0; q < L.ps; ++q)
        reinterpret_cast<uint64_t*>(ksim_smem + L.off_pk)[q * chunk + j] = c.ports[(int64_t)q * c.n + i];
    }
  }
  if (L.tables) {  // the pod-class tables (selector / toleration bits, reduce-class bytes)
    const int32_t C = c.n_classes_dev;
    for (int32_t k = tid; k < C * c.lwords; k += BS) reinterpret_cast<uint32_t*>(ksim_smem + L.off_sel)[k] = c.sel_ok[k];
    for (int32_t k = tid; k < C * c.twords; k += BS) {
      reinterpret_cast<uint32_t*>(ksim_smem + L.off_tok)[k] = c.taint_ok[k];
      reinterpret_cast<uint32_t*>(ksim_smem + L.off_nok)[k] = c.noexec_ok[k];
    }
    for (int32_t k = tid; k < C * c.n_taint_sets; k += BS) (ksim_smem + L.off_ttc)[k] = (char)c.tt_class[k];
    for (int32_t k = tid; k < C * c.n_label_sets; k += BS) (ksim_smem + L.off_nac)[k] = (char)c.na_class[k];
    for (int32_t k = tid; k < C * KSIM_MAX_RCLASS; k += BS) {
      reinterpret_cast<int64_t*>(ksim_smem + L.off_ttv)[k] = c.tt_val[k];
      reinterpret_cast<int64_t*>(ksim_smem + L.off_nav)[k] = c.na_val[k];
    }
  }
  if (tid == 0) { s_L = L; s_ctx = c; }
  // pod ring: RING_FILL descriptors (1 KiB) per refill, one 16-byte load per lane of wave 1
  // pod ring: RING_FILL descriptors (1 KiB) per refill, one 16-byte load per lane of wave 1.
  // The reduce-class counts k1 (TaintToleration) / k2 (NodeAffinity) ride in each queued
  // descriptor's reserved[0..1] (written by the library, ksim_launch_pod_k).
  auto ring_load = [&](int64_t p0, uint4& v) {
    const int64_t p = p0 + lane / 8;
    if (p < c.end) v = reinterpret_cast<const uint4*>(&c.pods[p])[lane % 8];
  };
  auto ring_store = [&](int64_t p0, const uint4& v) {
    const int64_t p = p0 + lane / 8;
    if (p < c.end) reinterpret_cast<uint4*>(&s_pod[p % RING])[lane % 8] = v;
  };
  if (wv == 1) {
    uint4 v;
    ring_load(c.first, v);
    ring_store(c.first, v);
  }
  if (tid == 0) { s_fix[c.first & 1][0] = -1; s_arr = 0; }
  uint64_t counter = *c.counter;  // replicated genericScheduler.lastNodeIndex (control wave)
  __syncthreads();

  auto pod_K = [&](const ksim_pod& P) -> int { return P.reserved[0] * P.reserved[1]; };
  // one row against pod P → packed entry + reason mask (fast path when the pod qualifies)
  auto load_row = [&](int32_t j) -> KsimFastRow {
    KsimFastRow r;
    r.ac = R.ac[j]; r.am = R.am[j]; r.rc = R.rc[j]; r.rm = R.rm[j]; r.zc = R.zc[j]; r.zm = R.zm[j];
    r.dac = R.dac[j]; r.dam = R.dam[j];
    r.allowed = R.allowed[j]; r.count = R.count[j]; r.fl = R.fl[j];
    return r;
  };
  auto eval_one = [&](const ksim_pod& P, bool fast, int32_t j, uint32_t& rm) -> int32_t {
    if (fast) {
      const KsimFastPod F{P.req_cpu, P.req_mem, P.nz_cpu, P.nz_mem, P.flags};
      return ksim_fast_eval(preds, F, load_row(j), no_prio, wl, wmr, wb, rm);
    }
    const RowEval e = eval_row_general((lds_ctx*)&s_ctx, (lds_layout*)&s_L, (lds_pod*)&P, (int)chunk, lo + j, j);
    rm = e.rm;
    return ev_pack(e.fit != 0, e.cl, e.sc);
  };
  // row wave: all rows of this lane for pod p → LDS entries + reason masks
  auto eval_rows = [&](int64_t p, int32_t (&e)[NPT], uint32_t (&rm)[NPT], int32_t* ev) {
    const ksim_pod& P = s_pod[p % RING];
    const bool fast = ksim_is_fast_pod(P, pod_K(P));
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int32_t j = k * RT + rt;
      e[k] = -1;
      rm[k] = 0;
      if (j < nrows) {
        e[k] = eval_one(P, fast, j, rm[k]);
        ev[j] = e[k];
      }
    }
  };
  // (fit count, per-class max, count at max) of one row wave's entries → LDS slot w
  auto partial = [&](const int32_t (&e)[NPT], int K, int buf, int w) {
    uint64_t fm[NPT];
    int32_t nf = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      fm[k] = __ballot(e[k] >= 0);
      nf += __popcll(fm[k]);
    }
    if (K == 1) {  // class 0: the entry is the score
      int32_t v = -1;
#pragma unroll
      for (int k = 0; k < NPT; ++k) v = e[k] > v ? e[k] : v;
      const int32_t wm = ksimw::max_i32(v);
      int32_t n = 0;
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const uint64_t bm = wm < 0 ? 0ull : __ballot(e[k] == wm);
        n += __popcll(bm);
        if (lane == 0) { s_fm[buf][k][w] = fm[k]; s_bm[buf][k][w] = bm; }
      }
      if (lane == 0) { s_fit[buf][w] = nf; s_mx[buf][w][0] = wm; s_cnt[buf][w][0] = n; }
      return;
    }
    if (lane == 0) s_fit[buf][w] = nf;
    for (int q = 0; q < K; ++q) {
      int32_t v = -1;
#pragma unroll
      for (int k = 0; k < NPT; ++k)
        if (e[k] >= 0 && ev_cls(e[k]) == q && ev_score(e[k]) > v) v = ev_score(e[k]);
      const int32_t wm = ksimw::max_i32(v);
      int32_t n = 0;
#pragma unroll
      for (int k = 0; k < NPT; ++k) n += __popcll(__ballot(e[k] >= 0 && ev_cls(e[k]) == q && ev_score(e[k]) == wm));
      if (lane == 0) { s_mx[buf][w][q] = wm; s_cnt[buf][w][q] = (wm < 0) ? 0 : n; }
    }
  };
  // control wave: combine the row waves' partials → granule payloads (lane q = class q)
  auto combine = [&](int K, int buf) -> uint64_t {
    const int q = lane < K ? lane : 0;
    int32_t f = 0, mx[NW], cn[NW];
#pragma unroll
    for (int w = 1; w < NW; ++w) {  // all loads first: one LDS round trip
      f += s_fit[buf][w];
      mx[w] = s_mx[buf][w][q];
      cn[w] = s_cnt[buf][w][q];
    }
    int32_t m = -1, n = 0;
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      const bool up = cn[w] != 0 && mx[w] > m, eq = cn[w] != 0 && mx[w] == m;
      n = up ? cn[w] : (eq ? n + cn[w] : n);
      m = up ? mx[w] : m;
    }
    if (lane >= K) return 0;
    return (lane == 0 ? ((uint64_t)f << 44) : 0) | ((uint64_t)n << 32) | (uint64_t)(uint32_t)m;
  };
  auto ptag = [&](int64_t p) -> uint64_t { return (uint64_t)((p - c.first + 1) & 0xFF); };
  // row waves: the last one to finish pod p's partial combines and publishes it
  auto arrive_publish = [&](int64_t p, int K, int buf) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    int32_t old = 0;
    if (lane == 0) old = atomicAdd(&s_arr, 1);
    old = __builtin_amdgcn_readfirstlane(old);
    if ((old + 1) % (NW - 1) == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      const uint64_t v = combine(K, buf);
      if (lane < K) store_granule(spec_at(granules, (int)(p % NSLOT), blockIdx.x, lane), (ptag(p) << 56) | v);
    }
  };

  // ---- prologue: partial of the first pod ----
  uint32_t A_rm[NPT], B_rm[NPT];
  if (wv > 0) {
    int32_t e[NPT];
    const int K0 = pod_K(s_pod[c.first % RING]);
    eval_rows(c.first, e, A_rm, R.ev + (c.first & 1) * chunk);
    partial(e, K0, c.first & 1, wv);
    arrive_publish(c.first, K0, c.first & 1);
  }
  int X = -1;  // control wave: owner workgroup of the previous pod's node (-1: none)
  __syncthreads();
#ifdef KSIM_STAMPS
  uint64_t t_prev = __builtin_amdgcn_s_memtime();
#endif

  for (int64_t pod = c.first; pod < c.end; ++pod) {
    const bool has_next = pod + 1 < c.end;
    const int pb = (int)(pod & 1);        // LDS buffers of pod
    const int nb = (int)((pod + 1) & 1);  // LDS buffers of pod + 1
    int32_t jsel = -1;                    // control wave: row committed by this workgroup
    bool have_pre = false;                // ... and its pod + 1 evaluation, when computed early
    int32_t ej_pre = -1;
    uint32_t rm_pre = 0;
#ifdef KSIM_STAMPS
    uint64_t o_prev = 0;
#endif

    if (wv == 0) {
      const ksim_pod& P = s_pod[pod % RING];
      const int K = pod_K(P);
      const int k2 = P.reserved[1];
      // the reduce classes' map values (lane q = class q), loaded now, used after the sweep
      int64_t tv_l = 0, av_l = 0;
      if (K > 1 && lane < K) {
        const int64_t* ttv = L.tables ? reinterpret_cast<const int64_t*>(ksim_smem + L.off_ttv) : c.tt_val;
        const int64_t* nav = L.tables ? reinterpret_cast<const int64_t*>(ksim_smem + L.off_nav) : c.na_val;
        tv_l = ttv[(int64_t)P.cls * KSIM_MAX_RCLASS + lane / k2];
        av_l = nav[(int64_t)P.cls * KSIM_MAX_RCLASS + lane % k2];
      }
      // ---------------- a. sweep: every speculative partial of pod + the owner's correction ----
      const uint64_t tag = ptag(pod);
      const int slot = (int)(pod % NSLOT);
      STAMP(1);
      uint64_t g[MAXB];
      bool ok = false;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#ifdef KSIM_STAMPS
      bool seen_spec = false, seen_fix = false;
#endif
      for (;;) {
        // unconditional loads (slots are sized for MAXG workgroups): one fabric round trip for
        // class 0, the owner's correction and (KF at a time) the further reduce classes
#pragma unroll
        for (int j = 0; j < MAXB; ++j) g[j] = load_granule(spec_at(granules, slot, lane * MAXB + j, 0));
        const uint64_t fx = load_granule(fix_at(granules, slot, 0));
        bool mine = X < 0 || gtag(fx) == tag;
#pragma unroll
        for (int j = 0; j < MAXB; ++j) {
          const int b = lane * MAXB + j;
          mine &= (b >= G) || b == X || gtag(g[j]) == tag;
        }
        for (int q0 = 1; q0 < K; q0 += KF) {  // classes >= 1 were published with class 0
          uint64_t v[KF][MAXB];
#pragma unroll
          for (int u = 0; u < KF; ++u)
#pragma unroll
            for (int j = 0; j < MAXB; ++j) {
              const int b = lane * MAXB + j;
              v[u][j] = (q0 + u < K && b < G) ? load_granule(gran_at(granules, slot, b, q0 + u, X)) : 0;
            }
#pragma unroll
          for (int u = 0; u < KF; ++u)
#pragma unroll
            for (int j = 0; j < MAXB; ++j) {
              const int b = lane * MAXB + j;
              if (q0 + u < K && b < G) {
                mine &= gtag(v[u][j]) == tag;
                s_gq[q0 + u - 1][b] = v[u][j];
              }
            }
        }
#ifdef KSIM_STAMPS
        st_acc[8] += 1;
        {
          bool sp = true;
#pragma unroll
          for (int j = 0; j < MAXB; ++j) sp &= (lane * MAXB + j >= G) || lane * MAXB + j == X || gtag(g[j]) == tag;
          const uint64_t tn = __builtin_amdgcn_s_memtime();
          if (!seen_spec && __all(sp)) { seen_spec = true; st_acc[12] += tn - t_prev; }
          if (!seen_fix && (X < 0 || gtag(fx) == tag)) { seen_fix = true; st_acc[13] += tn - t_prev; }
        }
#endif
        if (__all(mine)) {
          ok = true;
#pragma unroll
          for (int j = 0; j < MAXB; ++j) g[j] = (lane * MAXB + j == X) ? fx : g[j];
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_LIMIT_TICKS) break;
        __builtin_amdgcn_s_sleep(1);
      }
      STAMP(2);
#pragma unroll
      for (int j = 0; j < MAXB; ++j) g[j] = (lane * MAXB + j < G) ? g[j] : 0;
      ok = __all(ok);
      int32_t F = 0, M0 = -1, C0 = 0;
      if (ok) {
        int32_t f = 0, m = -1, n = 0;
#pragma unroll
        for (int j = 0; j < MAXB; ++j) {
          f += gfit(g[j]);
          const int32_t cnt = gcnt(g[j]), s = gscore(g[j]);
          if (cnt == 0) continue;
          if (s > m) { m = s; n = cnt; }
          else if (s == m) n += cnt;
        }
        F = ksimw::sum_i32(f);
        M0 = ksimw::max_i32(n ? m : -1);
        C0 = ksimw::sum_i32((n && m == M0) ? n : 0);
      }
      STAMP(9);
      if (ok && K > 1) {  // further reduce classes (TaintToleration x NodeAffinity), swept above
        if (lane == 0) { s_M[0] = M0; s_C[0] = C0; }
        for (int q = 1; q < K; ++q) {
          int32_t mm = -1, nn = 0;
#pragma unroll
          for (int j = 0; j < MAXB; ++j) {
            const int b = lane * MAXB + j;
            if (b >= G) continue;
            const uint64_t v = s_gq[q - 1][b];
            const int32_t cnt = gcnt(v), s = gscore(v);
            if (cnt == 0) continue;
            if (s > mm) { mm = s; nn = cnt; }
            else if (s == mm) nn += cnt;
          }
          const int32_t Mq = ksimw::max_i32(nn ? mm : -1);
          const int32_t Cq = ksimw::sum_i32((nn && mm == Mq) ? nn : 0);
          if (lane == 0) { s_M[q] = Mq; s_C[q] = Cq; }
        }
      }
      STAMP(11);
      int mode = 0, blk = -1, rank = 0;
      uint32_t win = 1;
      if (!ok) {
        mode = -1;
        if (lane == 0) atomicOr(c.err, 4);
      } else if (F > 0) {
        mode = 1;
        int64_t ix = 0;
        if (F > 1) {  // generic_scheduler.go:153-156: a single fit skips selectHost
          mode = 2;
          int64_t C = C0;
          if (K > 1) {
            // lane q = reduce class q, all at once: NormalizeReduce's maxima over the filtered
            // set (classes with fit nodes), each class's weighted total, the best total and the
            // classes that reach it (reduce.go:29-64, generic_scheduler.go:632-639)
            const bool live = lane < K && s_C[lane < K ? lane : 0] != 0;
            const int32_t cq = live ? s_C[lane] : 0;
            const int64_t mq = live ? s_M[lane] : 0;
            const int64_t mxT = wave_max_i64(live ? tv_l : 0), mxA = wave_max_i64(live ? av_l : 0);
            const int64_t t = live ? class_total(c, tv_l, av_l, mq, mxT, mxA) : -1;  // totals are >= 0
            const int64_t best = wave_max_i64(t);
            const uint64_t wb = __ballot(live && t == best);
            win = (uint32_t)wb;
            C = ksimw::sum_i32((wb >> lane) & 1ull ? cq : 0);
          }
          ix = (counter >> 32) ? (int64_t)(counter % (uint64_t)C) : (int64_t)((uint32_t)counter % (uint32_t)C);
          counter += 1;  // generic_scheduler.go:192-195
        }
        STAMP(10);
        // ---- locate the workgroup holding the ix-th match counted from the top ----
        int32_t bm[MAXB];
        int32_t tot = 0;
#pragma unroll
        for (int j = 0; j < MAXB; ++j) {
          const int b = lane * MAXB + j;
          int32_t m = 0;
          if (b < G) {
            if (mode == 1) {
              m = gfit(g[j]);
            } else {
              if ((win & 1u) && gcnt(g[j]) && gscore(g[j]) == M0) m += gcnt(g[j]);
              for (int q = 1; q < K; ++q) {
                if (!((win >> q) & 1u)) continue;
                const uint64_t v = s_gq[q - 1][b];
                if (gcnt(v) && gscore(v) == s_M[q]) m += gcnt(v);
              }
            }
          }
          bm[j] = m;
          tot += m;
        }
        const int32_t pre = ksimw::prefix_incl_i32(tot);
        const int32_t total = __builtin_amdgcn_readlane(pre, 63);
        const int64_t above = (int64_t)(total - pre);  // matches in workgroups of higher lanes
        const bool hit = tot > 0 && ix >= above && ix < above + tot;
        int32_t found = -1, r = 0;
        if (hit) {
          int64_t rr = ix - above;
#pragma unroll
          for (int j = MAXB - 1; j >= 0; --j) {
            if (found < 0) {
              if (rr < bm[j]) found = lane * MAXB + j;
              else rr -= bm[j];
            }
          }
          r = (int32_t)rr;
        }
        const uint64_t hb = __ballot(hit);
        if (hb == 0) {
          mode = -1;
        } else {
          const int src = __builtin_ffsll((long long)hb) - 1;
          blk = __builtin_amdgcn_readlane(found, src);
          rank = __builtin_amdgcn_readlane(r, src);
          if (blk < 0) mode = -1;
        }
        if (mode < 0 && lane == 0) atomicOr(c.err, 2);
      }
      STAMP(3);
#ifdef KSIM_STAMPS
      o_prev = __builtin_amdgcn_s_memtime();
#endif
      if (mode > 0 && blk == (int)blockIdx.x) {
        // ---------------- d. owner: exact row (rank from the top), commit ----------------
        if (K == 1) {
          // lane t = t-th 64-row segment from the top (k descending, then wave descending)
          constexpr int S = NPT * (NW - 1);
          uint64_t m = 0;
          if (lane < S) {
            const int k = NPT - 1 - lane / (NW - 1), w = NW - 1 - lane % (NW - 1);
            m = (mode == 1) ? s_fm[pb][k][w] : (s_mx[pb][w][0] == M0 ? s_bm[pb][k][w] : 0ull);
          }
          const int32_t cnt = __popcll(m);
          const int32_t pre = ksimw::prefix_incl_i32(cnt);
          const uint64_t hm = __ballot(pre > rank);
          if (hm) {
            const int ts = __builtin_ffsll((long long)hm) - 1;
            const int32_t r2 = rank - (__builtin_amdgcn_readlane(pre, ts) - __builtin_amdgcn_readlane(cnt, ts));
            const uint64_t ms = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(m >> 32), ts) << 32) |
                                (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)m, ts);
            // the r2-th set bit counted from the top: set, with exactly r2 set bits above it
            const bool is = ((ms >> lane) & 1ull) && __popcll((ms >> lane) >> 1) == r2;
            const uint64_t bb = __ballot(is);
            if (bb) {
              const int ks = NPT - 1 - ts / (NW - 1), ws = NW - 1 - ts % (NW - 1);
              jsel = ks * RT + (ws - 1) * 64 + (__builtin_ffsll((long long)bb) - 1);
            }
          }
        } else {  // several reduce classes: scan the packed entries from the top
          const int32_t* ev = R.ev + pb * chunk;
          int32_t rr = rank;
          const int nseg = (nrows + 63) / 64;
          for (int s0 = nseg - 1; s0 >= 0 && jsel < 0; s0 -= 4) {
            uint64_t bl[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int32_t j = (s0 - u) * 64 + lane;
              const int32_t e = (s0 - u >= 0 && j < nrows) ? ev[j] : -1;
              bool mt = e >= 0;
              if (mode == 2 && mt) {
                const int q = ev_cls(e);
                mt = ((win >> q) & 1u) && ev_score(e) == (q == 0 ? M0 : s_M[q]);
              }
              bl[u] = __ballot(mt);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              if (jsel >= 0) break;
              uint64_t m = bl[u];
              const int nbits = __popcll(m);
              if (rr >= nbits) { rr -= nbits; continue; }
              for (int t = 0; t < rr; ++t) m &= ~(1ull << (63 - __clzll(m)));
              jsel = (s0 - u) * 64 + (63 - __clzll(m));
            }
          }
        }
        OSTAMP(22);
        if (jsel < 0) {
          mode = -1;
          if (lane == 0) atomicOr(c.err, 2);
        } else {
          // commit (NodeInfo.AddPod); the committed row stays in registers for the fix-up
          KsimFastRow r = load_row(jsel);
          r.rc += P.add_cpu; r.rm += P.add_mem; r.zc += P.nz_cpu; r.zm += P.nz_mem; r.count += 1;
          const bool side = (P.add_gpu | P.add_eph | P.scalar_cnt | P.port_cnt) != 0;
          if (lane == 0) {
            R.rc[jsel] = r.rc; R.rm[jsel] = r.rm; R.zc[jsel] = r.zc; R.zm[jsel] = r.zm; R.count[jsel] = r.count;
            if (side) {
              const bool lds_ports = P.port_cnt && L.ps;
              if (P.add_gpu | P.add_eph | P.scalar_cnt | (P.port_cnt && !L.ps)) {
                r.fl = commit_side(cg, &P, lo + jsel, r.fl, lds_ports ? 0 : 1);
                R.fl[jsel] = r.fl;
              }
              if (lds_ports) commit_ports_lds(cg, &P, lo + jsel, jsel, (int32_t)chunk, L.off_pc, L.off_pk);
            }
            c.out_node[pod] = (int32_t)(lo + jsel);
          }
          OSTAMP(23);
          if (has_next) {  // pod + 1 against the committed row, before the barrier
            const ksim_pod& Q = s_pod[(pod + 1) % RING];
            const int Kq = pod_K(Q);
            if (ksim_is_fast_pod(Q, Kq) && !side) {
              const KsimFastPod F{Q.req_cpu, Q.req_mem, Q.nz_cpu, Q.nz_mem, Q.flags};
              ej_pre = ksim_fast_eval(preds, F, r, no_prio, wl, wmr, wb, rm_pre);
              have_pre = true;
            } else if (!ksim_is_fast_pod(Q, Kq)) {
              // general pod: everything it reads is in LDS; lane 0's commit stores first
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
              ej_pre = eval_one(Q, false, jsel, rm_pre);
              have_pre = true;
            }
          }
        }
        OSTAMP(16);
      }
      if (mode == 0 && blockIdx.x == 0 && lane == 0) c.out_node[pod] = -1;
      if (lane == 0) s_mode = mode;
      X = mode > 0 ? blk : -1;
      STAMP(6);
    } else {
      // ---------------- b. speculative evaluation of pod + 1 (row waves) ----------------
      // wave 1 refills the descriptor ring every RING_FILL pods; the load's latency hides
      // under the evaluation, the LDS store lands before the next barrier
      const bool refill = wv == 1 && ((pod - c.first) % RING_FILL) == 0;
      uint4 rv;
      if (refill) ring_load(pod + RING_FILL, rv);
#ifdef KSIM_STAMPS
      const uint64_t te0 = __builtin_amdgcn_s_memtime();
#endif
      if (has_next) {
        int32_t e[NPT];
        const int Kn = pod_K(s_pod[(pod + 1) % RING]);
        eval_rows(pod + 1, e, B_rm, R.ev + nb * chunk);
#ifdef KSIM_STAMPS
        const uint64_t te1 = __builtin_amdgcn_s_memtime();
        if (tid == 64) st_acc[14] += te1 - te0;
#endif
        partial(e, Kn, nb, wv);
#ifdef KSIM_STAMPS
        const uint64_t te2 = __builtin_amdgcn_s_memtime();
        if (tid == 64) st_acc[15] += te2 - te1;
#endif
        arrive_publish(pod + 1, Kn, nb);
      }
#ifdef KSIM_STAMPS
      if (tid == 64) st_acc[5] += __builtin_amdgcn_s_memtime() - te0;
#endif
      if (refill) ring_store(pod + RING_FILL, rv);
    }
    __syncthreads();
    STAMP(7);
    const int mode = s_mode;
    if (mode < 0) break;  // uniform: every workgroup reaches the same verdict

    if (mode == 0 && c.collect && c.out_reasons) {  // FitError: every workgroup adds its reasons
      if (tid < KSIM_NREASONS) s_hist[tid] = 0;
      __syncthreads();
      if (wv > 0) {
        const int32_t fr = s_fix[pb][0];
        const uint32_t fm = (uint32_t)s_fix[pb][1];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const uint32_t rm = (k * RT + rt == fr) ? fm : A_rm[k];
          for (int r = 0; r < KSIM_NREASONS; ++r) {
            const int32_t n = __popcll(__ballot((rm >> r) & 1u));
            if (lane == 0 && n) atomicAdd(&s_hist[r], n);
          }
        }
      }
      __syncthreads();
      if (tid < KSIM_NREASONS && s_hist[tid]) atomicAdd(&c.out_reasons[pod * KSIM_NREASONS + tid], s_hist[tid]);
    }
    if (wv == 0 && has_next) {
      // ---------------- e. owner: fix-up of pod + 1, publish the correction ----------------
      if (jsel >= 0) {  // only row jsel changed: re-evaluate it and redo its row wave's partial
        OSTAMP(17);
        const ksim_pod& Q = s_pod[(pod + 1) % RING];
        const int Kn = pod_K(Q);
        uint32_t rmj = rm_pre;
        const int32_t ej = have_pre ? ej_pre : eval_one(Q, ksim_is_fast_pod(Q, Kn), jsel, rmj);
        OSTAMP(18);
        const int w = 1 + (jsel % RT) / 64;
        int32_t e[NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int32_t j = k * RT + (w - 1) * 64 + lane;
          e[k] = (j == jsel) ? ej : (j < nrows ? R.ev[nb * chunk + j] : -1);
        }
        partial(e, Kn, nb, w);
        if (lane == 0) { R.ev[nb * chunk + jsel] = ej; s_fix[nb][0] = jsel; s_fix[nb][1] = (int32_t)rmj; }
        OSTAMP(19);
        const uint64_t v = combine(Kn, nb);
        if (lane < Kn) store_granule(fix_at(granules, (int)((pod + 1) % NSLOT), lane), (ptag(pod + 1) << 56) | v);
        OSTAMP(20);
#ifdef KSIM_STAMPS
        if (lane == 0) atomicAdd((unsigned long long*)&c.dbg[21], 1ull);
#endif
      } else if (lane == 0) {
        s_fix[nb][0] = -1;
      }
    }
    STAMP(4);
    if (wv > 0) {
#pragma unroll
      for (int k = 0; k < NPT; ++k) A_rm[k] = B_rm[k];
    }
  }

  // the table is authoritative in HBM between calls: write the owned rows back
  __syncthreads();
  for (int32_t j = tid; j < nrows; j += BS) {
    const int64_t i = lo + j;
    c.req_cpu[i] = R.rc[j]; c.req_mem[i] = R.rm[j];
    c.nz_cpu[i] = R.zc[j]; c.nz_mem[i] = R.zm[j];
    c.pod_count[i] = R.count[j]; c.flags[i] = R.fl[j];
  }
  if (blockIdx.x == 0 && tid == 0) {
    *c.counter = counter;
    *c.cursor = c.end;
  }
#ifdef KSIM_STAMPS
  if (blockIdx.x == 0 && tid == 0)
    for (int k = 0; k < 16; ++k) c.dbg[k] += (k == 5) ? 0 : st_acc[k];
  if (blockIdx.x == 0 && tid == 64) { c.dbg[5] += st_acc[5]; c.dbg[24] += st_acc[14]; c.dbg[25] += st_acc[15]; }
#endif
}

// Checks the DPP wave helpers against plain lane loops (diagnostic, tests/ only).
__global__ void ksim_wave_selftest_kernel(int32_t* out) {
  const int lane = threadIdx.x;
  const int32_t v = (int32_t)((lane * 7919 + 13) % 97) - 40 + (blockIdx.x * 11);
  out[(blockIdx.x * 3 + 0) * 64 + lane] = ksimw::max_i32(v);
  out[(blockIdx.x * 3 + 1) * 64 + lane] = ksimw::sum_i32(v);
  out[(blockIdx.x * 3 + 2) * 64 + lane] = ksimw::prefix_incl_i32(v);
}

// ---------------------------------------------------------------------------------------
static constexpr int LDS_BUDGET = 120 * 1024;

static int num_cus() {
  int dev = 0;
  hipDeviceProp_t p;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return 0;
  return p.multiProcessorCount;
}

// One workgroup per CU (<= 256) so every workgroup is resident — the protocol spins on every
// other workgroup — and chunk = ceil(n / grid) rows per workgroup held in LDS.
extern "C" int ksim_persistent_config(int64_t n, int* grid, int* lds_rows) {
  int g = num_cus();
  if (g <= 0 || n <= 0) return 0;
  if (g > 64 * MAXB) g = 64 * MAXB;
  if (n < (int64_t)g * 64) g = (int)((n + 63) / 64);  // >= 64 rows per workgroup
  if (g < 1) g = 1;
  const int64_t chunk = (n + g - 1) / g;
  if (chunk * LDS_ROW_BYTES > LDS_BUDGET || chunk > 4095 || chunk > 8 * 448) return 0;  // launch mode
  *grid = g;
  *lds_rows = (int)chunk;
  return 1;
}

extern "C" size_t ksim_persistent_granule_bytes(int) {
  return (size_t)(NSLOT * MAXG * GR + NSLOT * GR) * sizeof(uint64_t);
}

// Static LDS of the kernel instance (granule stash, rings, partials), for the dynamic budget.
template <int BS, int NPT>
static size_t static_lds() {
  hipFuncAttributes fa;
  if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&ksim_persistent_kernel<BS, NPT>)) != hipSuccess) return 48 * 1024;
  return fa.sharedSizeBytes;
}

template <int BS, int NPT>
static hipError_t launch_persistent(const KsimCtx* c, const KsimCtx* cdev, uint64_t* granules, int grid, int lds_rows,
                                    hipStream_t s) {
  const size_t lds_max = 160 * 1024 - static_lds<BS, NPT>();
  auto al = [](size_t b) { return (b + 15) & ~(size_t)15; };
  size_t off = al((size_t)lds_rows * LDS_ROW_BYTES);
  if (off > lds_max) return hipErrorInvalidValue;  // ksim_persistent_config keeps rows within budget
  PLayout L{};
  // the rows' host ports, when the node table has any and they fit
  const size_t pbytes = al((size_t)lds_rows * 4) + al((size_t)lds_rows * 8 * c->port_slots);
  if (c->port_slots > 0 && off + pbytes <= lds_max) {
    L.ps = c->port_slots;
    L.off_pc = (int32_t)off;
    L.off_pk = (int32_t)(off + al((size_t)lds_rows * 4));
    off += pbytes;
  }
  // the pod-class tables, when they fit
  const size_t C = (size_t)c->n_classes_dev;
  const size_t tb = al(C * c->lwords * 4) + 2 * al(C * c->twords * 4) + al(C * c->n_taint_sets) + al(C * c->n_label_sets) +
                    2 * al(C * KSIM_MAX_RCLASS * 8);
  if (C > 0 && off + tb <= lds_max) {
    L.tables = 1;
    L.off_sel = (int32_t)off; off += al(C * c->lwords * 4);
    L.off_tok = (int32_t)off; off += al(C * c->twords * 4);
    L.off_nok = (int32_t)off; off += al(C * c->twords * 4);
    L.off_ttc = (int32_t)off; off += al(C * c->n_taint_sets);
    L.off_nac = (int32_t)off; off += al(C * c->n_label_sets);
    L.off_ttv = (int32_t)off; off += al(C * KSIM_MAX_RCLASS * 8);
    L.off_nav = (int32_t)off; off += al(C * KSIM_MAX_RCLASS * 8);
  }
  hipLaunchKernelGGL((ksim_persistent_kernel<BS, NPT>), dim3(grid), dim3(BS), off, s, *c, cdev, granules, L);
  return hipGetLastError();
}

extern "C" hipError_t ksim_launch_persistent(const KsimCtx* c, const KsimCtx* cdev, uint64_t* granules, int grid,
                                             int lds_rows, hipStream_t s) {
  if (lds_rows <= 448) return launch_persistent<512, 1>(c, cdev, granules, grid, lds_rows, s);
  if (lds_rows <= 896) return launch_persistent<512, 2>(c, cdev, granules, grid, lds_rows, s);
  if (lds_rows <= 1792) return launch_persistent<512, 4>(c, cdev, granules, grid, lds_rows, s);
  return launch_persistent<512, 8>(c, cdev, granules, grid, lds_rows, s);
}

extern "C" int ksim_selftest(void) {
  int32_t* d = nullptr;
  const int nb = 4;
  if (hipMalloc(&d, nb * 3 * 64 * sizeof(int32_t)) != hipSuccess) return -1;
  hipLaunchKernelGGL(ksim_wave_selftest_kernel, dim3(nb), dim3(64), 0, 0, d);
  int32_t h[nb * 3 * 64];
  int bad = -1;
  if (hipDeviceSynchronize() == hipSuccess && hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) == hipSuccess) {
    bad = 0;
    for (int b = 0; b < nb; ++b) {
      int32_t v[64], mx = INT32_MIN, sum = 0, pre = 0;
      for (int l = 0; l < 64; ++l) {
        v[l] = (int32_t)((l * 7919 + 13) % 97) - 40 + b * 11;
        mx = v[l] > mx ? v[l] : mx;
        sum += v[l];
      }
      for (int l = 0; l < 64; ++l) {
        pre += v[l];
        bad += h[(b * 3 + 0) * 64 + l] != mx;
        bad += h[(b * 3 + 1) * 64 + l] != sum;
        bad += h[(b * 3 + 2) * 64 + l] != pre;
      }
    }
  }
  (void)hipFree(d);
  return bad;
}
