// ksim_pipe.hip — the two-deep pipelined form of the fast persistent kernel (resource-only
// pods, map-only policies, one device): the C3 headline path.
//
// Same cycle as ksim_pfast.hip (findNodesThatFit + PrioritizeNodes + selectHost + AddPod per pod,
// core/generic_scheduler.go:112-198, 542-676; least_requested.go:36-53,
// balanced_resource_allocation.go:39-61, node_info.go:318-341), same float64 arithmetic
// (ksim_f64.h), same cached evaluations (per (tree class, row) in LDS, only the committed row
// re-evaluated), but the per-pod cross-CU hand-off is taken off the critical path:
//
//  * Every workgroup b owns a name-rank range, and a pod's decision needs every workgroup's
//    (fit count, max score, count at max).  For pod q those statistics depend on the commits of
//    pods < q; a commit changes one row, so for every b except the owner of pod q-1 they are the
//    "spec" statistics of b's rows after pod q-2's commit.  The owner of q-1 differs only by one
//    row: its statistics are the spec ones with that row's evaluation replaced.
//  * So after deciding pod q-2 and applying its commit, workgroup b publishes for pod q:
//      A_b(q) = (fit, count at max, max)  and  B_b(q) = (second max, its count),
//      F_b(q)[r] = (e_old, e_new, stop) for every rank r of b's candidate rows for pod q-1 —
//    the rows at b's maximum of pod q-1, ranked from the top as selectHost ranks them — where
//    e_old / e_new are pod q's evaluation of that row before / after pod q-1 is committed to it.
//  * The decision of pod q (made redundantly by every workgroup's control wave) reads A(q) of
//    every workgroup and, for the owner X and rank r of pod q-1's decision, B_X(q) and
//    F_X(q)[r], and applies the O(1) correction.  Those were published a whole decision earlier,
//    so the per-pod critical path is one load of already-visible words plus the decision, not a
//    publish → observe hand-off: two decisions are in flight at once.
//
// Roles in a 512-thread workgroup: wave 0 decides (no barrier, no LDS rows); waves 1-7 own the
// rows: after decision q they commit pod q (owner only: NodeInfo.AddPod on the LDS row and the
// row's evaluation for every class), publish A/B(q+2), rank the candidate rows of pod q+1 and
// publish F(q+2).  Waves synchronise through LDS sequence words only.  Every spin is bounded.
#include <algorithm>

#include "ksim_f64.h"
#include "ksim_tree.h"
#include "ksim_wave.h"

using namespace kf64;

namespace {

constexpr int BS = 512;
constexpr int RW = BS / 64 - 1;  // row waves
constexpr int RT = RW * 64;      // row threads
constexpr int MAXB = 4;          // workgroups per sweep lane (grid <= 256)
constexpr int MAXG = 64 * MAXB;
constexpr int NSLOT = 8;         // pod slots of the published words (pod mod NSLOT)
constexpr int NREP = 8;          // replicas of A (workgroup b polls replica b % NREP)
constexpr int REP_STRIDE = NSLOT * MAXG + 64;
constexpr int DR = 8;            // decision ring (LDS)
constexpr int SR = 4;            // statistics ring (LDS, pod mod SR)
constexpr int RING = 32;         // pod-descriptor ring (LDS)
constexpr int RING_FILL = 8;
constexpr uint64_t SPIN_LIMIT_TICKS = 200000000ull;  // s_memrealtime at 100 MHz = 2 s
constexpr double EXACT_LIM = 281474976710656.0;     // 2^48

typedef __attribute__((address_space(1))) uint64_t gu64;
__device__ __forceinline__ void gstore(uint64_t* g, uint64_t v) {
  __hip_atomic_store((gu64*)g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t gload(const uint64_t* g) {
  return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// LDS sequence words between the waves of one workgroup
__device__ __forceinline__ void seq_release(int32_t* s, int32_t v) {
  __hip_atomic_store(s, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int32_t seq_acquire(int32_t* s) {
  return __hip_atomic_load(s, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// A: tag:8 | fit:13 | count:13 | score:29 (two's complement, -1 = no fit row)
__device__ __forceinline__ uint32_t gtag(uint64_t v) { return (uint32_t)(v >> 56); }
__device__ __forceinline__ int32_t gfit(uint64_t v) { return (int32_t)((v >> 42) & 0x1FFF); }
__device__ __forceinline__ int32_t gcnt(uint64_t v) { return (int32_t)((v >> 29) & 0x1FFF); }
__device__ __forceinline__ int32_t gscore(uint64_t v) { return ((int32_t)((uint32_t)v << 3)) >> 3; }
__device__ __forceinline__ uint64_t apack(uint64_t tag, int32_t f, int32_t n, int32_t m) {
  return (tag << 56) | ((uint64_t)(uint32_t)f << 42) | ((uint64_t)(uint32_t)n << 29) | ((uint64_t)(uint32_t)m & 0x1FFFFFFFull);
}
// B: tag:8 | m2:16 (signed) | c2:16
__device__ __forceinline__ uint64_t bpack(uint64_t tag, int32_t m2, int32_t c2) {
  return (tag << 56) | ((uint64_t)(uint16_t)(int16_t)m2 << 16) | (uint64_t)(uint16_t)c2;
}
__device__ __forceinline__ int32_t bm2(uint64_t v) { return (int32_t)(int16_t)(uint16_t)(v >> 16); }
__device__ __forceinline__ int32_t bc2(uint64_t v) { return (int32_t)(uint16_t)v; }
// F: tag:8 | stop:1 | e_old:16 (signed) | e_new:16 (signed)
__device__ __forceinline__ uint64_t fpack(uint64_t tag, bool stop, int32_t eo, int32_t en) {
  return (tag << 56) | ((uint64_t)stop << 55) | ((uint64_t)(uint16_t)(int16_t)eo << 16) | (uint64_t)(uint16_t)(int16_t)en;
}
__device__ __forceinline__ bool fstop(uint64_t v) { return (v >> 55) & 1; }
__device__ __forceinline__ int32_t feo(uint64_t v) { return (int32_t)(int16_t)(uint16_t)(v >> 16); }
__device__ __forceinline__ int32_t fen(uint64_t v) { return (int32_t)(int16_t)(uint16_t)v; }

// The owner's statistics after one of its rows goes from evaluation eo to en (top-two form;
// the same formula in the deciding control waves and in the owner's row waves).
struct Stat3 {
  int32_t f, c, m;
};
__device__ __forceinline__ Stat3 fix_stats(int32_t f, int32_t m1, int32_t c1, int32_t m2, int32_t c2, int32_t eo,
                                           int32_t en) {
  const bool rem = eo >= 0, add = en >= 0;
  const int32_t c1a = c1 - ((rem && eo == m1) ? 1 : 0);
  const int32_t mb = c1a ? m1 : (c2 ? m2 : -1), cb = c1a ? c1a : c2;
  const bool up = add && (cb == 0 || en > mb), eq = add && !up && en == mb;
  Stat3 s;
  s.m = up ? en : mb;
  s.c = up ? 1 : cb + (eq ? 1 : 0);
  s.f = f - (rem ? 1 : 0) + (add ? 1 : 0);
  if (!s.c) s.m = -1;
  return s;
}

__device__ __forceinline__ bool past(uint64_t t0) { return __builtin_amdgcn_s_memrealtime() - t0 > SPIN_LIMIT_TICKS; }

}  // namespace

struct PpArgs {
  int64_t n, chunk, first, end;
  const int64_t* alloc_cpu;
  const int64_t* alloc_mem;
  const int32_t* allowed_pods;
  const uint32_t* flags;
  int64_t* req_cpu;
  int64_t* req_mem;
  int64_t* nz_cpu;
  int64_t* nz_mem;
  int32_t* pod_count;
  const ksim_pod* pods;
  const int32_t* tcls;
  const KsimTreeClass* tclass;
  int32_t ncls;
  uint64_t* counter;
  int64_t* cursor;
  int32_t* out_node;
  int32_t* out_reasons;
  int32_t* err;
  uint64_t* dbg;
  uint64_t* words;  // A replicas, then B [NSLOT][MAXG], then F [NSLOT][G][chunk]
  uint32_t preds;
  int32_t no_prio, collect;
  int32_t wl, wm, wb;
};

namespace {

struct PRows {
  double *ac, *am, *rc, *rm, *zc, *zm, *yc, *ym;
  int32_t *allowed, *count;
  uint32_t* fl;
  int16_t* cache;  // [ncls][chunk]
};
constexpr int PP_ROW_BYTES = 8 * 8 + 3 * 4;  // 76 + the cache

extern __shared__ __attribute__((aligned(16))) char kp_smem[];

__device__ __forceinline__ PRows pcarve(int rows) {
  PRows r;
  double* d = reinterpret_cast<double*>(kp_smem);
  r.ac = d; r.am = d + rows; r.rc = d + 2 * rows; r.rm = d + 3 * rows;
  r.zc = d + 4 * rows; r.zm = d + 5 * rows; r.yc = d + 6 * rows; r.ym = d + 7 * rows;
  int32_t* q = reinterpret_cast<int32_t*>(d + 8 * rows);
  r.allowed = q; r.count = q + rows;
  r.fl = reinterpret_cast<uint32_t*>(q + 2 * rows);
  r.cache = reinterpret_cast<int16_t*>(q + 3 * rows + (rows & 1));  // 8-byte aligned
  return r;
}

__device__ __forceinline__ FRow prow(const PRows& R, int32_t j) {
  FRow r;
  r.ac = R.ac[j]; r.am = R.am[j]; r.rc = R.rc[j]; r.rm = R.rm[j]; r.zc = R.zc[j]; r.zm = R.zm[j];
  r.yc = R.yc[j]; r.ym = R.ym[j];
  r.allowed = R.allowed[j]; r.count = R.count[j]; r.fl = R.fl[j];
  return r;
}

}  // namespace

template <int NPT>
__global__ __launch_bounds__(BS) void ksim_pipe_kernel(PpArgs a) {
  __shared__ int32_t s_wst[SR][RW][5];  // per row wave: fit, m1, c1, m2, c2 (pod mod SR)
  __shared__ int32_t s_wg[SR][5];       // the workgroup's spec statistics of the pod
  __shared__ int32_t s_wg_seq[SR];      // relative pod index the slot holds (merged)
  __shared__ int32_t s_arr[SR];         // row waves arrived at the slot's merge
  __shared__ int32_t s_dec[DR][3];      // decision: mode, owner workgroup, rank
  __shared__ int32_t s_dec_seq;         // last decided relative pod
  __shared__ int32_t s_commit_seq;      // last relative pod committed by this workgroup (or -1)
  __shared__ int32_t s_m1next;          // the owner's max of the next pod after its commit
  __shared__ int32_t s_iter_done;       // row-wave iterations finished (sum over the waves)
  __shared__ int32_t s_stop;            // a row wave hit its spin bound
  __shared__ __attribute__((aligned(16))) ksim_pod s_pod[RING];
  __shared__ int32_t s_pcls[RING];
  __shared__ KsimTreeClass s_tcl[KSIM_TREE_MAX_CLASSES];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int rt = tid - 64;
  const int G = gridDim.x;
  const int me = blockIdx.x;
  const int64_t chunk = a.chunk;
  const int64_t lo = (int64_t)me * chunk;
  const int64_t hi = (lo + chunk < a.n) ? lo + chunk : a.n;
  const int32_t nrows = (int32_t)(hi - lo);
  const PRows R = pcarve((int)chunk);
  const EvCfg EC = make_evcfg(a.preds, a.no_prio != 0, a.wl, a.wm, a.wb);
  uint64_t* const Aw = a.words;
  uint64_t* const Bw = a.words + NREP * REP_STRIDE;
  uint64_t* const Fw = Bw + NSLOT * MAXG;
  const int64_t first = a.first, end = a.end;
  const int32_t npods = (int32_t)(end - first);
  auto ptag = [&](int32_t rel) -> uint64_t { return (uint64_t)((rel + 1) & 0xFF); };
  // the first spin that hit its bound: workgroup, wave, site, pod (and a site-specific value)
  auto note = [&](int site, int32_t rel, int32_t aux) {
    if (lane == 0)
      atomicCAS((unsigned long long*)a.dbg, 0ull,
                ((unsigned long long)me << 52) | ((unsigned long long)wv << 48) | ((unsigned long long)site << 40) |
                    ((unsigned long long)(aux & 0xFFFF) << 24) | (unsigned long long)(rel & 0xFFFFFF));
  };
  auto aslot = [&](uint64_t* base, int32_t rel, int b) -> uint64_t* {
    return base + (rel % NSLOT) * MAXG + (b % MAXB) * 64 + b / MAXB;
  };
  auto fslot = [&](int32_t rel, int b, int32_t r) -> uint64_t* {
    return Fw + ((int64_t)(rel % NSLOT) * G + b) * chunk + r;
  };

  // ---- stage the rows, the class inputs and the first pods; every class's evaluations ----
  for (int32_t j = tid; j < nrows; j += BS) {
    const int64_t i = lo + j;
    const double ac = (double)a.alloc_cpu[i], am = (double)a.alloc_mem[i];
    R.ac[j] = ac; R.am[j] = am;
    R.yc[j] = ac != 0.0 ? 1.0 / ac : 0.0;
    R.ym[j] = am != 0.0 ? 1.0 / am : 0.0;
    R.rc[j] = (double)a.req_cpu[i]; R.rm[j] = (double)a.req_mem[i];
    R.zc[j] = (double)a.nz_cpu[i]; R.zm[j] = (double)a.nz_mem[i];
    R.allowed[j] = a.allowed_pods[i]; R.count[j] = a.pod_count[i]; R.fl[j] = a.flags[i];
  }
  for (int k = tid; k < a.ncls; k += BS) s_tcl[k] = a.tclass[k];
  for (int x = tid; x < 2 * RING_FILL * 8 && first + x / 8 < end; x += BS) {  // pods [first, first + 16)
    const int64_t p = first + x / 8;
    reinterpret_cast<uint4*>(&s_pod[p % RING])[x % 8] = reinterpret_cast<const uint4*>(&a.pods[p])[x % 8];
  }
  for (int x = tid; x < 2 * RING_FILL && first + x < end; x += BS) s_pcls[(first + x) % RING] = a.tcls[first + x];
  if (tid < SR) { s_wg_seq[tid] = -1000; s_arr[tid] = 0; }
  if (tid == 0) { s_dec_seq = -1; s_commit_seq = -1; s_iter_done = 0; s_stop = 0; }
  __syncthreads();
  auto cls_fpod = [&](int k) -> FPod {
    const KsimTreeClass& t = s_tcl[k];
    return FPod{t.rq_c, t.rq_m, t.nz_c, t.nz_m, 0.0, 0.0, t.anyreq, t.be};
  };
  {
    const int tot = a.ncls * nrows;
    for (int idx = tid; idx < tot; idx += BS) {
      const int k = idx / nrows, j = idx - k * nrows;
      uint32_t rm;
      R.cache[k * chunk + j] = (int16_t)feval(EC, cls_fpod(k), prow(R, j), rm);
    }
  }
  __syncthreads();

  // ---------------- row-wave work ----------------
  const int w = wv;  // row wave 1..RW
  // spec statistics of pod rel (class c) over the rows as they stand: wave partials, the last
  // arriving wave merges, stores the workgroup's top two in s_wg and publishes A and B
  auto spec_publish = [&](int32_t rel) {
    const int c = s_pcls[(first + rel) % RING];
    const int16_t* cc = R.cache + (int64_t)c * chunk;
    int32_t e[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int32_t j = k * RT + rt;
      e[k] = j < nrows ? (int32_t)cc[j] : -1;
    }
    int32_t v = -1, nf = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      nf += __popcll(__ballot(e[k] >= 0));
      v = e[k] > v ? e[k] : v;
    }
    const int32_t m1 = ksimw::max_i32(v);
    int32_t v2 = -1;
#pragma unroll
    for (int k = 0; k < NPT; ++k) v2 = (e[k] < m1 && e[k] > v2) ? e[k] : v2;
    const int32_t m2 = ksimw::max_i32(v2);
    int32_t c1 = 0, c2 = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      c1 += m1 < 0 ? 0 : __popcll(__ballot(e[k] == m1));
      c2 += m2 < 0 ? 0 : __popcll(__ballot(e[k] == m2));
    }
    const int sl = rel % SR;
    if (lane == 0) {
      s_wst[sl][w - 1][0] = nf; s_wst[sl][w - 1][1] = m1; s_wst[sl][w - 1][2] = c1;
      s_wst[sl][w - 1][3] = m2; s_wst[sl][w - 1][4] = c2;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    int32_t old = 0;
    if (lane == 0) old = atomicAdd(&s_arr[sl], 1);
    old = __builtin_amdgcn_readfirstlane(old);
    if (old + 1 == RW) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
      const bool in = lane < RW;
      const int x = in ? lane : 0;
      const int32_t f = in ? s_wst[sl][x][0] : 0;
      const int32_t a1 = s_wst[sl][x][1], n1 = in ? s_wst[sl][x][2] : 0;
      const int32_t a2 = s_wst[sl][x][3], n2 = in ? s_wst[sl][x][4] : 0;
      const int32_t tf = ksimw::sum_i32(f);
      const int32_t tm1 = ksimw::max_i32(n1 ? a1 : -1);
      const int32_t tc1 = ksimw::sum_i32((n1 && a1 == tm1) ? n1 : 0);
      const int32_t tm2 = ksimw::max_i32(n1 && a1 < tm1 ? a1 : (n2 ? a2 : -1));
      int32_t tc2 = ksimw::sum_i32(((n1 && a1 == tm2) ? n1 : 0) + ((n2 && a2 == tm2) ? n2 : 0));
      if (tm2 < 0) tc2 = 0;
      if (lane == 0) s_arr[sl] = 0;  // before the publish: the slot's next use follows it
      const uint64_t tg = ptag(rel);
      if (lane < NREP) gstore(aslot(Aw + lane * REP_STRIDE, rel, me), apack(tg, tf, tc1, tm1));
      if (lane == NREP) gstore(Bw + (rel % NSLOT) * MAXG + me, bpack(tg, tm2, tc2));
      if (lane == 0) {
        s_wg[sl][0] = tf; s_wg[sl][1] = tm1; s_wg[sl][2] = tc1; s_wg[sl][3] = tm2; s_wg[sl][4] = tc2;
        seq_release(&s_wg_seq[sl], rel);
      }
    }
  };
  // wait until the merged statistics of pod rel are in s_wg (false: spin bound)
  auto wait_wg = [&](int32_t rel) -> bool {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (seq_acquire(&s_wg_seq[rel % SR]) != rel) {
      if (past(t0)) { note(1, rel, seq_acquire(&s_wg_seq[rel % SR])); return false; }
      __builtin_amdgcn_s_sleep(1);
    }
    return true;
  };
  // candidate rows of pod rel1 (rows at this workgroup's maximum M1, ranked from the top) and,
  // for each, pod rel1 + 1's evaluation before / after pod rel1 is committed to it → F
  uint64_t tmask[NPT];  // this wave's candidate rows of the pod being decided next, per segment
  int32_t tabove[NPT];  // candidates in the segments above each
  auto rank_and_fix = [&](int32_t rel1, int32_t M1) {
    const int c1 = s_pcls[(first + rel1) % RING];
    const int16_t* cc = R.cache + (int64_t)c1 * chunk;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int32_t j = k * RT + rt;
      tmask[k] = __ballot(M1 >= 0 && j < nrows && (int32_t)cc[j] == M1);
      int32_t n = 0;
      if (M1 >= 0)
        for (int32_t x = k * RT + w * 64 + lane; x < nrows; x += 64) n += ((int32_t)cc[x] == M1) ? 1 : 0;
      tabove[k] = ksimw::sum_i32(n);
    }
    const int32_t rel2 = rel1 + 1;
    if (rel2 >= npods) return;
    const ksim_pod& P1 = s_pod[(first + rel1) % RING];
    const FPod F1 = load_fpod(P1);
    const FPod F2 = load_fpod(s_pod[(first + rel2) % RING]);
    const int16_t* c2 = R.cache + (int64_t)s_pcls[(first + rel2) % RING] * chunk;
    const uint64_t tg = ptag(rel2);
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      if ((tmask[k] >> lane) & 1ull) {
        const int32_t j = k * RT + rt;
        const int32_t rank = tabove[k] + __popcll((tmask[k] >> lane) >> 1);
        const FRow r2 = plus(prow(R, j), F1);
        uint32_t m;
        const int32_t en = feval(EC, F2, r2, m);
        const bool stop = r2.rc >= EXACT_LIM || r2.rm >= EXACT_LIM || r2.zc >= EXACT_LIM || r2.zm >= EXACT_LIM;
        gstore(fslot(rel2, me, rank), fpack(tg, stop, (int32_t)c2[j], en));
      }
    }
  };

  int64_t stop_at = end;
#ifdef KSIM_STAMPS
  uint64_t st[8] = {};  // per wave: phase cycles summed over the pods (flushed at the end)
  uint64_t tp = __builtin_amdgcn_s_memtime();
#define PSTAMP(k)                                        \
  do {                                                   \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();    \
    st[k] += t_ - tp;                                    \
    tp = t_;                                             \
  } while (0)
#else
#define PSTAMP(k) do { } while (0)
#endif
  uint64_t counter = *a.counter;  // replicated genericScheduler.lastNodeIndex (control wave)

  if (wv > 0) {
    // ---- prologue: A/B of the first two pods, candidates of the first, F of the second ----
    spec_publish(0);
    bool ok = wait_wg(0);
    if (npods > 1) spec_publish(1);
    if (ok) rank_and_fix(0, s_wg[0][1]);
    uint4 ring_next = make_uint4(0, 0, 0, 0);  // wave 1: descriptors of the next refill
    int32_t ring_next_cl = 0;
    auto ring_load = [&](int64_t p0, uint4& v, int32_t& cl) {
      const int64_t p = p0 + lane / 8;
      if (p < end) v = reinterpret_cast<const uint4*>(&a.pods[p])[lane % 8];
      if (lane < RING_FILL && p0 + lane < end) cl = a.tcls[p0 + lane];
    };
    auto ring_store = [&](int64_t p0, const uint4& v, int32_t cl) {
      const int64_t p = p0 + lane / 8;
      if (p < end) reinterpret_cast<uint4*>(&s_pod[p % RING])[lane % 8] = v;
      if (lane < RING_FILL && p0 + lane < end) s_pcls[(p0 + lane) % RING] = cl;
    };
    if (wv == 1) ring_load(first + 2 * RING_FILL, ring_next, ring_next_cl);
    if (lane == 0) atomicAdd(&s_iter_done, 1);  // the prologue counts as iteration -1

    // ---- row iterations: after decision rel ----
    PSTAMP(7);
    for (int32_t rel = 0; ok && rel < npods; ++rel) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (seq_acquire(&s_dec_seq) < rel) {
        if (past(t0) || seq_acquire(&s_stop)) { note(2, rel, seq_acquire(&s_dec_seq)); ok = false; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      if (!ok) break;
      PSTAMP(0);  // waiting for the decision
      const int32_t mode = s_dec[rel % DR][0], X = s_dec[rel % DR][1], rk = s_dec[rel % DR][2];
      if (mode < 0) break;
      if (wv == 1 && (rel % RING_FILL) == 0) {  // pods [rel + 16, rel + 24) into the ring
        const int64_t p0 = first + rel + 2 * RING_FILL;
        ring_store(p0, ring_next, ring_next_cl);
        ring_load(p0 + RING_FILL, ring_next, ring_next_cl);
      }
      const int64_t pod = first + rel;
      if (mode == 0 && a.collect && a.out_reasons) {
        // FitError: the pod against this wave's rows as they stand
        const FPod P = load_fpod(s_pod[pod % RING]);
        uint32_t rms[NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int32_t j = k * RT + rt;
          rms[k] = 0;
          if (j < nrows) (void)feval(EC, P, prow(R, j), rms[k]);
        }
        for (int r = 0; r < KSIM_NREASONS; ++r) {
          int32_t nr = 0;
#pragma unroll
          for (int k = 0; k < NPT; ++k) nr += __popcll(__ballot((rms[k] >> r) & 1u));
          if (lane == 0 && nr) atomicAdd(&a.out_reasons[pod * KSIM_NREASONS + r], nr);
        }
      }
      const bool has1 = rel + 1 < npods;
      int32_t M1 = -1;  // this workgroup's maximum of pod rel + 1
      if (mode == 2 && X == me) {
        // ---- owner: the rk-th candidate from the top; commit, re-evaluate its row ----
        int32_t seg = -1, bit = -1;
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int32_t cnt = __popcll(tmask[k]);
          if (rk >= tabove[k] && rk < tabove[k] + cnt) {
            const int32_t want = rk - tabove[k];
            const uint64_t hb = __ballot(((tmask[k] >> lane) & 1ull) && __popcll((tmask[k] >> lane) >> 1) == want);
            seg = k;
            bit = __builtin_ctzll(hb);
          }
        }
        if (seg >= 0) {
          const int32_t j = seg * RT + (w - 1) * 64 + bit;
          // every row wave must have finished the previous iteration (they read this row)
          const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
          while (seq_acquire(&s_iter_done) < RW * (rel + 1)) {
            if (past(t1)) { note(3, rel, seq_acquire(&s_iter_done)); ok = false; break; }
            __builtin_amdgcn_s_sleep(1);
          }
          const FRow r2 = plus(prow(R, j), load_fpod(s_pod[pod % RING]));
          int32_t eo = -1, en = -1;
          if (has1) {
            const int c1 = s_pcls[(pod + 1) % RING];
            eo = R.cache[(int64_t)c1 * chunk + j];
          }
          if (lane < a.ncls) {
            uint32_t m;
            R.cache[(int64_t)lane * chunk + j] = (int16_t)feval(EC, cls_fpod(lane), r2, m);
          }
          if (has1) {
            const int c1 = s_pcls[(pod + 1) % RING];
            uint32_t m;
            en = feval(EC, cls_fpod(c1), r2, m);
            ok = ok && wait_wg(rel + 1);
            const int sl = (rel + 1) % SR;
            const Stat3 s = fix_stats(s_wg[sl][0], s_wg[sl][1], s_wg[sl][2], s_wg[sl][3], s_wg[sl][4], eo, en);
            if (lane == 0) s_m1next = s.m;
          }
          if (lane == 0) {
            R.rc[j] = r2.rc; R.rm[j] = r2.rm; R.zc[j] = r2.zc; R.zm[j] = r2.zm; R.count[j] = r2.count;
            a.out_node[pod] = (int32_t)(lo + j);
            if (r2.rc >= EXACT_LIM || r2.rm >= EXACT_LIM || r2.zc >= EXACT_LIM || r2.zm >= EXACT_LIM) atomicOr(a.err, 8);
            seq_release(&s_commit_seq, rel);
          }
        } else {
          const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
          while (seq_acquire(&s_commit_seq) < rel) {
            if (past(t1)) { note(4, rel, rk); ok = false; break; }
            __builtin_amdgcn_s_sleep(1);
          }
        }
        if (has1) M1 = __builtin_amdgcn_readfirstlane(s_m1next);
      } else if (has1) {
        ok = ok && wait_wg(rel + 1);
        M1 = s_wg[(rel + 1) % SR][1];
      }
      if (!ok) break;
      PSTAMP(1);  // reasons, commit / waiting for it
      if (rel + 2 < npods) spec_publish(rel + 2);
      PSTAMP(2);
      if (has1) rank_and_fix(rel + 1, M1);
      PSTAMP(3);
      if (lane == 0) atomicAdd(&s_iter_done, 1);
    }
    if (!ok && lane == 0) { atomicOr(a.err, 2); atomicExch(&s_stop, 1); }
  } else {
    // ---------------- control wave: decide every pod ----------------
    int X = -1;       // owner workgroup of the previous pod's node (-1: none)
    int32_t XR = 0;   // ... and the rank it took
    const uint64_t* my_rep = Aw + (me % NREP) * REP_STRIDE;
    PSTAMP(7);
    uint64_t spins = 0;
    for (int32_t rel = 0; rel < npods; ++rel) {
      const uint64_t tag = ptag(rel);
      uint64_t g[MAXB], bx = 0, fx = 0;
      bool ok = false;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
#pragma unroll
        for (int j = 0; j < MAXB; ++j) g[j] = gload(my_rep + (rel % NSLOT) * MAXG + j * 64 + lane);
        if (X >= 0) {
          bx = gload(Bw + (rel % NSLOT) * MAXG + X);
          fx = gload(fslot(rel, X, XR));
        }
        bool mine = X < 0 || (gtag(bx) == tag && gtag(fx) == tag);
#pragma unroll
        for (int j = 0; j < MAXB; ++j) {
          const int b = lane * MAXB + j;
          mine &= (b >= G) || gtag(g[j]) == tag;
        }
        if (__all(mine)) { ok = true; break; }
#ifdef KSIM_STAMPS
        spins += 1;
#endif
        if (past(t0) || seq_acquire(&s_stop)) {
          int32_t miss = -1;
#pragma unroll
          for (int j = 0; j < MAXB; ++j)
            if (lane * MAXB + j < G && gtag(g[j]) != tag) miss = lane * MAXB + j;
          const uint64_t mb = __ballot(miss >= 0);
          const int32_t m0 = mb ? __builtin_amdgcn_readlane(miss, __builtin_ctzll(mb)) : (X >= 0 ? 1000 + X : 999);
          note(5, rel, m0);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      PSTAMP(0);  // sweep
      bool stop_any = false;
      if (ok && X >= 0) {  // the previous owner's statistics with its committed row corrected
        const int lx = X / MAXB, jx = X % MAXB;
        const uint64_t ax = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)g[jx], lx) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(g[jx] >> 32), lx) << 32);
        const Stat3 s = fix_stats(gfit(ax), gscore(ax), gcnt(ax), bm2(bx), bc2(bx), feo(fx), fen(fx));
        stop_any = fstop(fx);
        const int64_t xr = a.n - (int64_t)X * chunk;
        if (s.c > (xr < chunk ? xr : chunk) && lane == 0 && me == 0) {  // diagnostic: the corrected count exceeds the rows
          a.dbg[8] = (uint64_t)rel | ((uint64_t)X << 32);
          a.dbg[9] = ax; a.dbg[10] = bx; a.dbg[11] = fx; a.dbg[12] = (uint64_t)XR;
        }
#pragma unroll
        for (int j = 0; j < MAXB; ++j) g[j] = (lane * MAXB + j == X) ? apack(tag, s.f, s.c, s.m) : g[j];
      }
      // findNodesThatFit count, max score, selectHost (generic_scheduler.go:136-198)
      int32_t f = 0, lm = -1;
#pragma unroll
      for (int j = 0; j < MAXB; ++j) {
        g[j] = (lane * MAXB + j < G) ? g[j] : 0;
        f += gfit(g[j]);
        lm = (gcnt(g[j]) && gscore(g[j]) > lm) ? gscore(g[j]) : lm;
      }
      const int32_t F = ksimw::sum_i32(f);
      const int32_t M = ksimw::max_i32(lm);
      int32_t bm[MAXB], tot = 0;
#pragma unroll
      for (int j = 0; j < MAXB; ++j) {
        bm[j] = (gcnt(g[j]) && gscore(g[j]) == M) ? gcnt(g[j]) : 0;
        tot += bm[j];
      }
      const int32_t pre = ksimw::prefix_incl_i32(tot);
      const uint32_t C = (uint32_t)__builtin_amdgcn_readlane(pre, 63);
      const uint32_t Cs = C ? C : 1u;
      const int64_t ix = (counter >> 32) ? (int64_t)(counter % (uint64_t)Cs) : (int64_t)((uint32_t)counter % Cs);
      const int64_t above = (int64_t)C - pre;  // matches in workgroups of higher lanes
      const bool hit = tot > 0 && ix >= above && ix < above + tot;
      int32_t found = -1;
      int64_t rr = ix - above;
#pragma unroll
      for (int j = MAXB - 1; j >= 0; --j) {
        const bool here = found < 0 && rr < bm[j];
        found = here ? lane * MAXB + j : found;
        rr = (found < 0) ? rr - bm[j] : rr;
      }
      const uint64_t hb = __ballot(hit);
      const int src = __builtin_ffsll((long long)hb) - 1;
      const int blk = hb ? __builtin_amdgcn_readlane(found, src) : -1;
      const int rank = hb ? __builtin_amdgcn_readlane((int32_t)rr, src) : 0;
      int mode;
      if (!ok) mode = -1;
      else if (stop_any) mode = -2;  // the previous commit left the exact float64 range
      else if (F == 0) mode = 0;
      else mode = (hb && blk >= 0) ? 2 : -1;
      if (mode == 2 && F > 1) counter += 1;  // generic_scheduler.go:192-195
      if (lane == 0) {
        if (mode == -1) atomicOr(a.err, ok ? 2 : 4);
        if (mode == 0 && me == 0) a.out_node[first + rel] = -1;
        s_dec[rel % DR][0] = mode; s_dec[rel % DR][1] = blk; s_dec[rel % DR][2] = rank;
        seq_release(&s_dec_seq, rel);
      }
      if (mode < 0) {
        if (mode == -2) stop_at = first + rel;
        break;
      }
      PSTAMP(1);  // decide
      X = mode == 2 ? blk : -1;
      XR = rank;
    }
#ifdef KSIM_STAMPS
    st[6] = spins;
#endif
  }
#ifdef KSIM_STAMPS
  if (lane == 0 && (wv == 0 || wv == 1 || wv == RW)) {  // summed over the workgroups: control, first and last row wave
    const int base = 16 + (wv == 0 ? 0 : wv == 1 ? 8 : 16);
    for (int k = 0; k < 8; ++k) atomicAdd((unsigned long long*)&a.dbg[base + k], st[k]);
  }
#endif
  // ---- the table is authoritative in HBM between calls: write the owned rows back ----
  __syncthreads();
  for (int32_t j = tid; j < nrows; j += BS) {
    const int64_t i = lo + j;
    a.req_cpu[i] = (int64_t)R.rc[j]; a.req_mem[i] = (int64_t)R.rm[j];
    a.nz_cpu[i] = (int64_t)R.zc[j]; a.nz_mem[i] = (int64_t)R.zm[j];
    a.pod_count[i] = R.count[j];
  }
  if (me == 0 && tid == 0) {
    *a.counter = counter;
    *a.cursor = stop_at;
  }
}

// ---------------------------------------------------------------------------------------
static constexpr int PP_LDS_BUDGET = 150 * 1024;

// LDS bytes of the pipelined kernel for lds_rows rows and ncls classes (0: does not fit)
extern "C" size_t ksim_pipe_lds_bytes(int lds_rows, int ncls) {
  if (ncls <= 0 || ncls > KSIM_TREE_MAX_CLASSES || lds_rows <= 0 || lds_rows > 4 * RT) return 0;
  const size_t b = (size_t)lds_rows * PP_ROW_BYTES + 8 + (size_t)ncls * lds_rows * 2;
  return b <= (size_t)PP_LDS_BUDGET ? ((b + 15) & ~(size_t)15) : 0;
}

// words: A replicas, B, F [NSLOT][grid][lds_rows]
extern "C" size_t ksim_pipe_word_bytes(int grid, int lds_rows) {
  return ((size_t)NREP * REP_STRIDE + (size_t)NSLOT * MAXG + (size_t)NSLOT * grid * lds_rows) * sizeof(uint64_t);
}

extern "C" hipError_t ksim_launch_pipe(const KsimCtx* c, uint64_t* words, int grid, int lds_rows, const int32_t* tcls,
                                       const KsimTreeClass* tclass, int ncls, hipStream_t s) {
  const size_t lds = ksim_pipe_lds_bytes(lds_rows, ncls);
  if (!lds || grid <= 0 || grid > MAXG || (int64_t)grid * lds_rows < c->n) return hipErrorInvalidValue;
  PpArgs a;
  a.n = c->n; a.chunk = lds_rows; a.first = c->first; a.end = c->end;
  a.alloc_cpu = c->alloc_cpu; a.alloc_mem = c->alloc_mem; a.allowed_pods = c->allowed_pods; a.flags = c->flags;
  a.req_cpu = c->req_cpu; a.req_mem = c->req_mem; a.nz_cpu = c->nz_cpu; a.nz_mem = c->nz_mem;
  a.pod_count = c->pod_count; a.pods = c->pods; a.tcls = tcls; a.tclass = tclass; a.ncls = ncls;
  a.counter = c->counter; a.cursor = c->cursor;
  a.out_node = c->out_node; a.out_reasons = c->out_reasons; a.err = c->err; a.dbg = c->dbg; a.words = words;
  a.preds = c->preds; a.no_prio = c->no_prio; a.collect = c->collect;
  a.wl = (int32_t)c->w[KSIM_W_LEAST_REQUESTED]; a.wm = (int32_t)c->w[KSIM_W_MOST_REQUESTED];
  a.wb = (int32_t)c->w[KSIM_W_BALANCED];
#define KSIM_PP(R)                                                              \
  do {                                                                          \
    hipError_t e_ = ksim_check_coresident(ksim_pipe_kernel<R>, grid, BS, lds);  \
    if (e_ != hipSuccess) return e_;                                            \
    hipLaunchKernelGGL((ksim_pipe_kernel<R>), dim3(grid), dim3(BS), lds, s, a); \
  } while (0)
  if (lds_rows <= RT) KSIM_PP(1);
  else if (lds_rows <= 2 * RT) KSIM_PP(2);
  else KSIM_PP(4);
#undef KSIM_PP
  return hipGetLastError();
}
