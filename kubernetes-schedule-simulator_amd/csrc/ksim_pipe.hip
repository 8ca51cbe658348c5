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
//    so two decisions are in flight at once: pod q's decision waits for the row work that
//    followed pod q-2's, not for the one that follows pod q-1's.
//  * The per-pod row work is O(1) statistics plus the candidates' re-evaluations: every
//    workgroup keeps, per class, a histogram of its rows' cached scores (workgroup-wide and per
//    64-row segment; scores are small integers, < 64 bins), so A / B are two ballots over one
//    histogram, a wave finds the candidates above its segment from the segment histograms, and a
//    commit moves one row's entry in each class's histograms.
//  * The control wave's decision splits around the owner's words: the pre-decision over every
//    workgroup but the owner (sums, maxima, prefix counts) runs while B_X / F_X are loading, the
//    post-decision that adds the owner back is O(1).
//
// Roles in a 512-thread workgroup: wave 0 decides (no barrier, no LDS rows); waves 1-7 own the
// rows: after decision q they commit pod q (owner only: NodeInfo.AddPod on the LDS row, the
// row's evaluation for every class, the histograms), publish A/B(q+2) (wave 7), rank the
// candidate rows of pod q+1 and publish F(q+2).  Waves synchronise through LDS sequence words
// only.  Every spin is bounded.
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
// revision bit of A / B (bit 55) and F (bit 54) words: 0 = published speculatively before the
// decision of pod q-2 (as if this workgroup did not get pod q-2), 1 = republished by the owner of
// pod q-2 after its commit.  A decider knows pod q-2's owner, so it knows which revision to take.
__device__ __forceinline__ uint64_t arev(uint64_t v) { return (v >> 55) & 1; }
__device__ __forceinline__ uint64_t frev(uint64_t v) { return (v >> 54) & 1; }
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
  int32_t nb;  // score bins: every map score is in [0, nb), nb <= 64
  int32_t spec;  // 1: row work for pod rel + 2 is done before decision rel (revision bits); 0: after it
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
  int16_t* cache;  // [ncls][chunk]: class k's evaluation of row j as it stands (-1: does not fit)
  int32_t* hseg;   // [ncls][nseg][nb]: rows of 64-row segment s whose class-k evaluation is score b
  int32_t* hwg;    // [ncls][nb]: the same over the workgroup's rows
  int32_t* fitc;   // [ncls]: rows that fit class k
};
constexpr int PP_ROW_BYTES = 8 * 8 + 3 * 4;  // 76, then the cache and the histograms

extern __shared__ __attribute__((aligned(16))) char kp_smem[];

__device__ __forceinline__ PRows pcarve(int rows, int ncls, int nseg, int nb) {
  PRows r;
  double* d = reinterpret_cast<double*>(kp_smem);
  r.ac = d; r.am = d + rows; r.rc = d + 2 * rows; r.rm = d + 3 * rows;
  r.zc = d + 4 * rows; r.zm = d + 5 * rows; r.yc = d + 6 * rows; r.ym = d + 7 * rows;
  int32_t* q = reinterpret_cast<int32_t*>(d + 8 * rows);
  r.allowed = q; r.count = q + rows;
  r.fl = reinterpret_cast<uint32_t*>(q + 2 * rows);
  int32_t* h = q + 3 * rows;
  r.hseg = h;
  r.hwg = h + ncls * nseg * nb;
  r.fitc = r.hwg + ncls * nb;
  r.cache = reinterpret_cast<int16_t*>(r.fitc + ncls);
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

// LDS state shared by the two roles (the kernel arguments are copied here once: the role
// functions are kept out of line, each with its own register allocation)
struct PipeSh {
  PpArgs a;
  int32_t dec[DR][3];      // decision: mode, owner workgroup, rank
  int32_t dec_seq;         // last decided relative pod
  int32_t commit_seq;      // last relative pod committed by this workgroup (or -1)
  int32_t iter_done;       // row-wave iterations finished (sum over the waves)
  int32_t stop;            // a wave hit its spin bound
  uint64_t counter;        // the control wave's lastNodeIndex at the end
  int64_t stop_at;         // first pod not scheduled
  __attribute__((aligned(16))) ksim_pod pod[RING];
  int32_t pcls[RING];
  KsimTreeClass tcl[KSIM_TREE_MAX_CLASSES];
};

namespace {

__device__ __forceinline__ uint64_t ptag(int32_t rel) { return (uint64_t)((rel + 1) & 0xFF); }

// the first spin that hit its bound: workgroup, wave, site, pod (and a site-specific value)
__device__ __forceinline__ void note(const PpArgs& a, int site, int32_t rel, int32_t aux) {
  if ((threadIdx.x & 63) == 0)
    atomicCAS((unsigned long long*)a.dbg, 0ull,
              ((unsigned long long)blockIdx.x << 52) | ((unsigned long long)(threadIdx.x >> 6) << 48) |
                  ((unsigned long long)site << 40) | ((unsigned long long)(aux & 0xFFFF) << 24) |
                  (unsigned long long)(rel & 0xFFFFFF));
}

__device__ __forceinline__ uint64_t* aslot(uint64_t* base, int32_t rel, int b) {
  return base + (rel % NSLOT) * MAXG + (b % MAXB) * 64 + b / MAXB;
}
__device__ __forceinline__ uint64_t* bword(const PpArgs& a, int32_t rel, int b) {
  return a.words + NREP * REP_STRIDE + (rel % NSLOT) * MAXG + b;
}
__device__ __forceinline__ uint64_t* fslot(const PpArgs& a, int32_t rel, int b, int32_t r) {
  return a.words + NREP * REP_STRIDE + NSLOT * MAXG + ((int64_t)(rel % NSLOT) * gridDim.x + b) * a.chunk + r;
}

__device__ __forceinline__ FPod cls_fpod(const PipeSh& S, int k) {
  const KsimTreeClass& t = S.tcl[k];
  return FPod{t.rq_c, t.rq_m, t.nz_c, t.nz_m, 0.0, 0.0, t.anyreq, t.be};
}

}  // namespace

#ifdef KSIM_STAMPS
#define PSTAMP(k)                                     \
  do {                                                \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    st[k] += t_ - tp;                                 \
    tp = t_;                                          \
  } while (0)
#define PFLUSH(base)                                                                                   \
  do {                                                                                                 \
    if ((threadIdx.x & 63) == 0)                                                                       \
      for (int k_ = 0; k_ < 8; ++k_) atomicAdd((unsigned long long*)&a.dbg[(base) + k_], st[k_]);      \
  } while (0)
#else
#define PSTAMP(k) do { } while (0)
#define PFLUSH(base) do { } while (0)
#endif

// ---------------- row waves (1..RW) ----------------
template <int NPT>
__device__ __noinline__ void pipe_rows(PipeSh* Sp) {
  PipeSh& S = *Sp;
  const PpArgs& a = S.a;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rt = tid - 64;
  const int me = blockIdx.x;
  const int64_t chunk = a.chunk;
  const int64_t lo = (int64_t)me * chunk;
  const int32_t nrows = (int32_t)(((lo + chunk < a.n) ? lo + chunk : a.n) - lo);
  const int NB = a.nb, NSEG = (int)((chunk + 63) / 64), K = a.ncls;
  const PRows R = pcarve((int)chunk, K, NSEG, NB);
  const EvCfg EC = make_evcfg(a.preds, a.no_prio != 0, a.wl, a.wm, a.wb);
  const int64_t first = a.first, end = a.end;
  const int32_t npods = (int32_t)(end - first);
#ifdef KSIM_STAMPS
  uint64_t st[8] = {};
  uint64_t tp = __builtin_amdgcn_s_memtime();
#endif

  // the workgroup's (fit, max, count at max, second max, its count) for class c from the
  // histogram (lane b = bin b), published as A / B of pod rel by wave RW
  auto publish_ab = [&](int32_t rel, uint64_t rev) {
    const int c = S.pcls[(first + rel) % RING];
    const int32_t h = lane < NB ? R.hwg[c * NB + lane] : 0;
    const uint64_t nz = __ballot(h > 0);
    const int32_t m1 = nz ? 63 - __builtin_clzll(nz) : -1;
    const uint64_t nz2 = m1 >= 0 ? (nz & ~(1ull << m1)) : 0ull;
    const int32_t m2 = nz2 ? 63 - __builtin_clzll(nz2) : -1;
    const int32_t c1 = m1 >= 0 ? __builtin_amdgcn_readlane(h, m1) : 0;
    const int32_t c2 = m2 >= 0 ? __builtin_amdgcn_readlane(h, m2) : 0;
    const uint64_t tg = ptag(rel);
    if (lane < NREP) gstore(aslot(a.words + lane * REP_STRIDE, rel, me), apack(tg, R.fitc[c], c1, m1) | (rev << 55));
    if (lane == NREP) gstore(bword(a, rel, me), bpack(tg, m2, c2) | (rev << 55));
  };
  // candidate rows of pod rel1 (the rows at this workgroup's maximum of the pod's class, ranked
  // from the top) and, for each, pod rel1 + 1's evaluation before / after pod rel1 is committed
  // to it → F(rel1 + 1)
  uint64_t tmask[NPT];  // this wave's candidate rows of the pod being decided next, per segment
  int32_t tabove[NPT];  // candidates in the segments above each
  uint64_t tm_next[NPT];  // ... of the pod after it (the speculative / the owner's redo)
  int32_t ta_next[NPT];
  auto rank_and_fix = [&](int32_t rel1, uint64_t rev, uint64_t (&tmask)[NPT], int32_t (&tabove)[NPT]) {
    const int c1 = S.pcls[(first + rel1) % RING];
    const int32_t h = lane < NB ? R.hwg[c1 * NB + lane] : 0;
    const uint64_t nz = __ballot(h > 0);
    const int32_t M1 = nz ? 63 - __builtin_clzll(nz) : -1;
    const int16_t* cc = R.cache + (int64_t)c1 * chunk;
    // candidates per segment (lane = segment); suffix sums give the segments above
    const int32_t sc = (M1 >= 0 && lane < NSEG) ? R.hseg[(c1 * NSEG + lane) * NB + M1] : 0;
    const int32_t incl = ksimw::prefix_incl_i32(sc);
    const int32_t total = __builtin_amdgcn_readlane(incl, 63);
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int32_t j = k * RT + rt;
      tmask[k] = __ballot(M1 >= 0 && j < nrows && (int32_t)cc[j] == M1);
      tabove[k] = total - __builtin_amdgcn_readlane(incl, k * RW + w - 1);
    }
    const int32_t rel2 = rel1 + 1;
    if (rel2 >= npods) return;
    const FPod F1 = load_fpod(S.pod[(first + rel1) % RING]);
    const FPod F2 = load_fpod(S.pod[(first + rel2) % RING]);
    const int16_t* c2 = R.cache + (int64_t)S.pcls[(first + rel2) % RING] * chunk;
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
        gstore(fslot(a, rel2, me, rank), fpack(tg, stop, (int32_t)c2[j], en) | (rev << 54));
      }
    }
  };

  // ---- prologue: A/B of the first two pods, candidates of the first, F of the second ----
  if (w == RW) {
    publish_ab(0, 0);
    if (npods > 1) publish_ab(1, 0);
  }
  rank_and_fix(0, 0, tmask, tabove);
  bool ok = true;
  if (lane == 0) atomicAdd(&S.iter_done, 1);  // the prologue counts as iteration -1
  PSTAMP(7);

  // ---- row iterations ----
  // Before decision rel is known, every wave does pod rel + 2's work as if this workgroup does not
  // get pod rel (A / B(rel + 2), the candidates of pod rel + 1 and F(rel + 2), revision 0): only
  // pod rel's owner changes, and it redoes that work after its commit (revision 1).  So for every
  // workgroup but one the per-pod row work is off the critical path.
  for (int32_t rel = 0; rel < npods; ++rel) {
    if (a.spec && w == RW && rel + 2 < npods) publish_ab(rel + 2, 0);
    if (a.spec && rel + 1 < npods) rank_and_fix(rel + 1, 0, tm_next, ta_next);
    if (lane == 0) atomicAdd(&S.iter_done, 1);  // this iteration's speculative reads are done
    PSTAMP(2);  // the speculative work
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (seq_acquire(&S.dec_seq) < rel) {
      if (past(t0) || seq_acquire(&S.stop)) { note(a, 2, rel, seq_acquire(&S.dec_seq)); ok = false; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!ok) break;
    PSTAMP(0);  // waiting for the decision
    const int32_t mode = S.dec[rel % DR][0], X = S.dec[rel % DR][1], rk = S.dec[rel % DR][2];
    if (mode < 0) break;
    const bool own = mode == 2 && X == me;
    const int64_t pod = first + rel;
    if (mode == 0 && a.collect && a.out_reasons) {
      // FitError: the pod against this wave's rows as they stand
      const FPod P = load_fpod(S.pod[pod % RING]);
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
    if (own) {
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
        // every row wave must have finished this iteration's speculative reads (they read this row)
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        while (seq_acquire(&S.iter_done) < RW * (rel + 2)) {
          if (past(t1)) { note(a, 3, rel, seq_acquire(&S.iter_done)); ok = false; break; }
          __builtin_amdgcn_s_sleep(1);
        }
        const FRow r2 = plus(prow(R, j), load_fpod(S.pod[pod % RING]));
        if (lane < K) {  // the row's evaluation for every class, and the histograms
          uint32_t m;
          const int32_t eo = R.cache[(int64_t)lane * chunk + j];
          const int32_t en = feval(EC, cls_fpod(S, lane), r2, m);
          R.cache[(int64_t)lane * chunk + j] = (int16_t)en;
          const int sg = j >> 6;
          if (eo >= 0) {
            R.hseg[(lane * NSEG + sg) * NB + eo] -= 1;
            R.hwg[lane * NB + eo] -= 1;
          }
          if (en >= 0) {
            R.hseg[(lane * NSEG + sg) * NB + en] += 1;
            R.hwg[lane * NB + en] += 1;
          }
          R.fitc[lane] += (en >= 0 ? 1 : 0) - (eo >= 0 ? 1 : 0);
        }
        if (lane == 0) {
          R.rc[j] = r2.rc; R.rm[j] = r2.rm; R.zc[j] = r2.zc; R.zm[j] = r2.zm; R.count[j] = r2.count;
          a.out_node[pod] = (int32_t)(lo + j);
          if (r2.rc >= EXACT_LIM || r2.rm >= EXACT_LIM || r2.zc >= EXACT_LIM || r2.zm >= EXACT_LIM) atomicOr(a.err, 8);
        }
        seq_release(&S.commit_seq, rel);
      } else {
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        while (seq_acquire(&S.commit_seq) < rel) {
          if (past(t1)) { note(a, 4, rel, rk); ok = false; break; }
          __builtin_amdgcn_s_sleep(1);
        }
      }
    }
    if (!ok) break;
    if (own || !a.spec) {
      // pod rel + 2's work on the committed rows: the owner's redo (revision 1), or everyone's
      const uint64_t rv = a.spec ? 1ull : 0ull;
      if (w == RW && rel + 2 < npods) publish_ab(rel + 2, rv);
      if (rel + 1 < npods) rank_and_fix(rel + 1, rv, tm_next, ta_next);
    }
    PSTAMP(1);  // reasons, commit / waiting for it, the owner's redo
#pragma unroll
    for (int k = 0; k < NPT; ++k) { tmask[k] = tm_next[k]; tabove[k] = ta_next[k]; }
  }
  if (!ok && lane == 0) { atomicOr(a.err, 2); atomicExch(&S.stop, 1); }
  if (w == 1) PFLUSH(24);
  if (w == RW) PFLUSH(32);
}

// ---------------- control wave: decide every pod ----------------
// A(rel) of every workgroup is in g[] (lane l: workgroups 4l .. 4l+3); after each decision the
// loads of A(rel + 1) and of the owner's B / F words go out together, the pre-decision over
// every workgroup but the owner overlaps the owner's words, then an O(1) post-decision.
__device__ __noinline__ void pipe_control(PipeSh* Sp) {
  PipeSh& S = *Sp;
  const PpArgs& a = S.a;
  const int lane = threadIdx.x & 63;
  const int G = gridDim.x;
  const int me = blockIdx.x;
  const int64_t first = a.first;
  const int32_t npods = (int32_t)(a.end - first);
  // replicated genericScheduler.lastNodeIndex, uniform: read into scalar registers at once (a
  // vector register still pending from this load would make every later wait conservative)
  uint64_t counter;
  {
    const uint64_t c0 = *a.counter;
    counter = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(c0 >> 32)) << 32) |
              (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)c0);
  }
  int64_t stop_at = a.end;
#ifdef KSIM_STAMPS
  uint64_t st[8] = {};
  uint64_t tp = __builtin_amdgcn_s_memtime();
  uint64_t spins = 0;
#endif
  __builtin_amdgcn_s_setprio(2);  // the per-pod critical path: ahead of the row wave sharing this SIMD
  int X = -1;      // owner workgroup of the previous pod's node (-1: none)
  int32_t XR = 0;  // ... and the rank it took
  int X2 = -1;     // owner workgroup of the pod before that: its words of this pod are revision 1
  const uint64_t* my_rep = a.words + (me % NREP) * REP_STRIDE;
  uint64_t g[MAXB];
  // The pod-descriptor ring is refilled here, not by the row waves: a row wave that carried
  // prefetched descriptors across its loop would wait (s_waitcnt vmcnt(0), stores included) for
  // its own write-through stores at every iteration.  Every RING_FILL pods, pods [rel + 15,
  // rel + 23) go out with the A loads of pod rel and land in LDS once they are back (the row
  // waves read pods <= their pod + 2 and lag the decisions by <= 2 pods).
  // A(rel + 1) is prefetched once pod rel's owner words are in — by then the row work that
  // publishes it (after decision rel - 1) is normally done — so its load latency overlaps pod
  // rel's post-decision; a stale prefetch falls back to polling.
  uint64_t gn[MAXB];
  uint64_t rv0 = 0, rv1 = 0;  // a 16-byte quarter of a pod descriptor (lane / 8: pod, lane % 8: quarter)
  int32_t rcl = 0;
  const uint64_t* rq = reinterpret_cast<const uint64_t*>(a.pods);
  const int32_t* rt = a.tcls;
  bool pf_refill = false;
  int64_t pf_p0 = 0;
  // the prefetch's address stays live until its data is taken: a VGPR that addresses a load in
  // flight is not rewritten before the load returns (the compiler would wait for it there)
  const uint64_t* pf_addr = my_rep + lane;
  auto prefetch_a = [&](int32_t rel) {
    pf_refill = ((rel - 1) % RING_FILL) == 0;  // (rel >= 1: the prologue staged pods [first, first + 16))
    pf_p0 = first + rel + 2 * RING_FILL - 1;
    if (pf_refill) {  // (asm loads like the A prefetch below, waited for in take_a; clamped addresses)
      const int64_t pp = pf_p0 + lane / 8 < a.end ? pf_p0 + lane / 8 : a.end - 1;
      rq = reinterpret_cast<const uint64_t*>(&a.pods[pp]) + 2 * (lane % 8);
      rt = a.tcls + (pf_p0 + (lane % RING_FILL) < a.end ? pf_p0 + (lane % RING_FILL) : a.end - 1);
      asm volatile(
          "global_load_dwordx2 %0, %3, off\n\t"
          "global_load_dwordx2 %1, %3, off offset:8\n\t"
          "global_load_dword %2, %4, off"
          : "=&v"(rv0), "=&v"(rv1), "=&v"(rcl)
          : "v"(rq), "v"(rt)
          : "memory");
    }
    pf_addr = my_rep + (rel % NSLOT) * MAXG + lane;
    // the four A loads as one asm block: the compiler does not track them, so its conservative
    // waits in the post-decision (a 64-bit modulo, joins) do not wait for them; take_a waits
    // explicitly, with the destinations as in/out operands so nothing reads them earlier
    static_assert(MAXB == 4, "the prefetch asm loads four granules per lane");
    asm volatile(
        "global_load_dwordx2 %0, %4, off sc1\n\t"
        "global_load_dwordx2 %1, %4, off offset:512 sc1\n\t"
        "global_load_dwordx2 %2, %4, off offset:1024 sc1\n\t"
        "global_load_dwordx2 %3, %4, off offset:1536 sc1"
        : "=&v"(gn[0]), "=&v"(gn[1]), "=&v"(gn[2]), "=&v"(gn[3])
        : "v"(pf_addr)
        : "memory");
  };
  auto tags_ok = [&](const uint64_t (&v)[MAXB], uint64_t tag) -> bool {
    bool mine = true;
#pragma unroll
    for (int j = 0; j < MAXB; ++j) {
      const int b = lane * MAXB + j;
      mine &= (b >= G) || (gtag(v[j]) == tag && arev(v[j]) == (b == X2 ? 1ull : 0ull));
    }
    return __all(mine);
  };
  auto take_a = [&](int32_t rel) -> bool {  // the prefetched A(rel), or poll until every workgroup's is here
    const uint64_t tag = ptag(rel);
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(gn[0]), "+v"(gn[1]), "+v"(gn[2]), "+v"(gn[3]), "+v"(rv0), "+v"(rv1), "+v"(rcl)
                 : "v"(pf_addr), "v"(rq), "v"(rt) : "memory");
    if (pf_refill) {
      if (pf_p0 + lane / 8 < a.end) {
        uint64_t* d = reinterpret_cast<uint64_t*>(&S.pod[(pf_p0 + lane / 8) % RING]) + 2 * (lane % 8);
        d[0] = rv0;
        d[1] = rv1;
      }
      if (lane < RING_FILL && pf_p0 + lane < a.end) S.pcls[(pf_p0 + lane) % RING] = rcl;
    }
#pragma unroll
    for (int j = 0; j < MAXB; ++j) g[j] = gn[j];
    if (tags_ok(g, tag)) return true;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int j = 0; j < MAXB; ++j) g[j] = gload(pf_addr + j * 64);
      if (tags_ok(g, tag)) return true;
      if (past(t0) || seq_acquire(&S.stop)) {
        int32_t miss = -1;
#pragma unroll
        for (int j = 0; j < MAXB; ++j)
          if (lane * MAXB + j < G && (gtag(g[j]) != tag || arev(g[j]) != (lane * MAXB + j == X2 ? 1ull : 0ull)))
            miss = lane * MAXB + j;
        const uint64_t mb = __ballot(miss >= 0);
        note(a, 5, rel, mb ? __builtin_amdgcn_readlane(miss, __builtin_ctzll(mb)) : 999);
        return false;
      }
    }
  };
  PSTAMP(7);
  prefetch_a(0);
  bool ok = take_a(0);
  for (int32_t rel = 0; rel < npods; ++rel) {
    const uint64_t tag = ptag(rel);
    // the owner's words (address known since the last decision), in flight during the pre-decision
    uint64_t bx = 0, fx = 0;
    const uint64_t* pbx = bword(a, rel, X >= 0 ? X : 0);
    const uint64_t* pfx = fslot(a, rel, X >= 0 ? X : 0, XR);
    // (asm loads like the A prefetch: the compiler's conservative waits never hold them)
    auto owner_loads = [&]() {
      asm volatile("global_load_dwordx2 %0, %2, off sc1\n\tglobal_load_dwordx2 %1, %3, off sc1"
                   : "=&v"(bx), "=&v"(fx) : "v"(pbx), "v"(pfx) : "memory");
    };
    auto owner_wait = [&]() {
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(bx), "+v"(fx) : "v"(pbx), "v"(pfx) : "memory");
    };
    if (ok && X >= 0) owner_loads();
    // ---- pre-decision over every workgroup but X ----
    int32_t cnt[MAXB];
    int32_t f = 0, lm = -1;
#pragma unroll
    for (int j = 0; j < MAXB; ++j) {
      const int b = lane * MAXB + j;
      const bool v = b < G && b != X;
      f += v ? gfit(g[j]) : 0;
      lm = (v && gcnt(g[j]) && gscore(g[j]) > lm) ? gscore(g[j]) : lm;
    }
    const int32_t Fs = ksimw::sum_i32(f);
    const int32_t Ms = ksimw::max_i32(lm);
    int32_t tot = 0;
#pragma unroll
    for (int j = 0; j < MAXB; ++j) {
      const int b = lane * MAXB + j;
      cnt[j] = (b < G && b != X && gcnt(g[j]) && gscore(g[j]) == Ms) ? gcnt(g[j]) : 0;
      tot += cnt[j];
    }
    const int32_t pre = ksimw::prefix_incl_i32(tot);
    const int32_t Cs = __builtin_amdgcn_readlane(pre, 63);
    const int32_t abv = Cs - pre;  // matches in workgroups of higher lanes
    int32_t aboveX = 0;            // matches (at Ms) in workgroups above X
    uint64_t ax = 0;
    if (X >= 0) {
      const int lx = X / MAXB, jx = X % MAXB;
      int32_t part = 0;
#pragma unroll
      for (int j = 0; j < MAXB; ++j) part += j > jx ? cnt[j] : 0;
      aboveX = __builtin_amdgcn_readlane(abv + part, lx);
      ax = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)g[jx], lx) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(g[jx] >> 32), lx) << 32);
    }
    PSTAMP(2);  // pre-decision
    // ---- the owner's corrected statistics ----
    bool stop_any = false;
    int32_t fX = 0, cX = 0, mX = -1;
    if (ok && X >= 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      owner_wait();
      const uint64_t xrev = X == X2 ? 1ull : 0ull;  // (its words of this pod were redone after pod rel-2's commit)
      while (!(gtag(bx) == tag && gtag(fx) == tag && arev(bx) == xrev && frev(fx) == xrev)) {
        if (past(t0) || seq_acquire(&S.stop)) { note(a, 6, rel, X); ok = false; break; }
#ifdef KSIM_STAMPS
        spins += 1;
#endif
        __builtin_amdgcn_s_sleep(1);
        owner_loads();
        owner_wait();
      }
      const Stat3 s = fix_stats(gfit(ax), gscore(ax), gcnt(ax), bm2(bx), bc2(bx), feo(fx), fen(fx));
      fX = s.f; cX = s.c; mX = s.m;
      stop_any = fstop(fx);
    }
    PSTAMP(0);  // waiting for the owner's words
    if (rel + 1 < npods) prefetch_a(rel + 1);
    // ---- post-decision: findNodesThatFit count, max score, selectHost (generic_scheduler.go:136-198) ----
    const int32_t F = Fs + fX;
    const bool xtop = cX > 0 && (Cs == 0 || mX > Ms);  // X alone holds the maximum
    const bool xeq = cX > 0 && Cs > 0 && mX == Ms;      // X shares it
    const uint32_t C = (uint32_t)(xtop ? cX : Cs + (xeq ? cX : 0));
    const uint32_t Cd = C ? C : 1u;
    const int64_t ix = (counter >> 32) ? (int64_t)(counter % (uint64_t)Cd) : (int64_t)((uint32_t)counter % Cd);
    int blk = -1, rank = 0;
    int64_t t = ix;  // index among the other workgroups' matches, when X does not take it
    if (xtop) {
      blk = X; rank = (int)ix;
    } else if (xeq && ix >= aboveX && ix < aboveX + cX) {
      blk = X; rank = (int)(ix - aboveX);
    } else if (xeq && ix >= aboveX + cX) {
      t = ix - cX;
    }
    if (blk < 0 && C > 0) {
      const bool hit = tot > 0 && t >= abv && t < abv + tot;
      int32_t found = -1;
      int64_t rr = t - abv;
#pragma unroll
      for (int j = MAXB - 1; j >= 0; --j) {
        const bool here = found < 0 && rr < cnt[j];
        found = here ? lane * MAXB + j : found;
        rr = (found < 0) ? rr - cnt[j] : rr;
      }
      const uint64_t hb = __ballot(hit);
      if (hb) {
        const int src = __builtin_ctzll(hb);
        blk = __builtin_amdgcn_readlane(found, src);
        rank = __builtin_amdgcn_readlane((int32_t)rr, src);
      }
    }
    int mode;
    if (!ok) mode = -1;
    else if (stop_any) mode = -2;  // the previous commit left the exact float64 range
    else if (F == 0) mode = 0;
    else mode = blk >= 0 ? 2 : -1;
    if (mode == 2 && F > 1) counter += 1;  // generic_scheduler.go:192-195
    if (lane == 0) {
      if (mode == -1) atomicOr(a.err, ok ? 2 : 4);
      if (mode == 0 && me == 0) a.out_node[first + rel] = -1;
      S.dec[rel % DR][0] = mode; S.dec[rel % DR][1] = blk; S.dec[rel % DR][2] = rank;
      // release for the LDS words only (a full release would wait for the A prefetch in flight)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      __hip_atomic_store(&S.dec_seq, rel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    PSTAMP(1);  // post-decision
    if (mode < 0) {
      if (mode == -2) stop_at = first + rel;
      break;
    }
    X2 = a.spec ? X : -1;
    X = mode == 2 ? blk : -1;
    XR = rank;
    if (rel + 1 < npods) ok = take_a(rel + 1);
    PSTAMP(3);  // waiting for the next pod's A words
  }
  __builtin_amdgcn_s_setprio(0);
#ifdef KSIM_STAMPS
  st[6] = spins;
#endif
  PFLUSH(16);
  if (lane == 0) { S.counter = counter; S.stop_at = stop_at; }
}

template <int NPT>
__global__ __launch_bounds__(BS) void ksim_pipe_kernel(PpArgs a) {
  __shared__ PipeSh S;
  const int tid = threadIdx.x, wv = tid >> 6;
  const int me = blockIdx.x;
  const int64_t chunk = a.chunk;
  const int64_t lo = (int64_t)me * chunk;
  const int64_t hi = (lo + chunk < a.n) ? lo + chunk : a.n;
  const int32_t nrows = (int32_t)(hi - lo);
  const int NB = a.nb, NSEG = (int)((chunk + 63) / 64), K = a.ncls;
  const PRows R = pcarve((int)chunk, K, NSEG, NB);
  const EvCfg EC = make_evcfg(a.preds, a.no_prio != 0, a.wl, a.wm, a.wb);
  const int64_t first = a.first, end = a.end;

  // ---- stage the rows, the class inputs and the first pods ----
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
  for (int k = tid; k < K; k += BS) S.tcl[k] = a.tclass[k];
  for (int x = tid; x < 2 * RING_FILL * 8 && first + x / 8 < end; x += BS) {  // pods [first, first + 16)
    const int64_t p = first + x / 8;
    reinterpret_cast<uint4*>(&S.pod[p % RING])[x % 8] = reinterpret_cast<const uint4*>(&a.pods[p])[x % 8];
  }
  for (int x = tid; x < 2 * RING_FILL && first + x < end; x += BS) S.pcls[(first + x) % RING] = a.tcls[first + x];
  for (int x = tid; x < K * NSEG * NB + K * NB + K; x += BS) R.hseg[x] = 0;  // hseg, hwg, fitc are contiguous
  if (tid == 0) {
    S.a = a;
    S.dec_seq = -1; S.commit_seq = -1; S.iter_done = 0; S.stop = 0;
    S.counter = 0; S.stop_at = end;
  }
  __syncthreads();
  // every (class, owned row) evaluation, and the score histograms
  for (int idx = tid; idx < K * nrows; idx += BS) {
    const int k = idx / nrows, j = idx - k * nrows;
    uint32_t rm;
    const int32_t e = feval(EC, cls_fpod(S, k), prow(R, j), rm);
    R.cache[(int64_t)k * chunk + j] = (int16_t)e;
    if (e >= 0) {
      atomicAdd(&R.hseg[(k * NSEG + (j >> 6)) * NB + e], 1);
      atomicAdd(&R.hwg[k * NB + e], 1);
      atomicAdd(&R.fitc[k], 1);
    }
  }
  __syncthreads();

  if (wv > 0) pipe_rows<NPT>(&S);
  else pipe_control(&S);

  // ---- the table is authoritative in HBM between calls: write the owned rows back ----
  __syncthreads();
  for (int32_t j = tid; j < nrows; j += BS) {
    const int64_t i = lo + j;
    a.req_cpu[i] = (int64_t)R.rc[j]; a.req_mem[i] = (int64_t)R.rm[j];
    a.nz_cpu[i] = (int64_t)R.zc[j]; a.nz_mem[i] = (int64_t)R.zm[j];
    a.pod_count[i] = R.count[j];
  }
  if (me == 0 && tid == 0) {
    *a.counter = S.counter;
    *a.cursor = S.stop_at;
  }
}

// ---------------------------------------------------------------------------------------
static constexpr int PP_LDS_BUDGET = 150 * 1024;

// LDS bytes of the pipelined kernel for lds_rows rows, ncls classes and nb score bins (0: does not fit)
extern "C" size_t ksim_pipe_lds_bytes(int lds_rows, int ncls, int nb) {
  if (ncls <= 0 || ncls > KSIM_TREE_MAX_CLASSES || lds_rows <= 0 || lds_rows > 4 * RT || nb <= 0 || nb > 64) return 0;
  const size_t nseg = ((size_t)lds_rows + 63) / 64;
  const size_t b = (size_t)lds_rows * PP_ROW_BYTES + 4 * ((size_t)ncls * nseg * nb + (size_t)ncls * nb + ncls) +
                   (size_t)ncls * lds_rows * 2;
  return b <= (size_t)PP_LDS_BUDGET ? ((b + 15) & ~(size_t)15) : 0;
}

// words: A replicas, B, F [NSLOT][grid][lds_rows]
extern "C" size_t ksim_pipe_word_bytes(int grid, int lds_rows) {
  return ((size_t)NREP * REP_STRIDE + (size_t)NSLOT * MAXG + (size_t)NSLOT * grid * lds_rows) * sizeof(uint64_t);
}

extern "C" hipError_t ksim_launch_pipe(const KsimCtx* c, uint64_t* words, int grid, int lds_rows, int spec, const int32_t* tcls,
                                       const KsimTreeClass* tclass, int ncls, int nb, hipStream_t s) {
  const size_t lds = ksim_pipe_lds_bytes(lds_rows, ncls, nb);
  if (!lds || grid <= 0 || grid > MAXG || (int64_t)grid * lds_rows < c->n) return hipErrorInvalidValue;
  PpArgs a;
  a.n = c->n; a.chunk = lds_rows; a.first = c->first; a.end = c->end;
  a.alloc_cpu = c->alloc_cpu; a.alloc_mem = c->alloc_mem; a.allowed_pods = c->allowed_pods; a.flags = c->flags;
  a.req_cpu = c->req_cpu; a.req_mem = c->req_mem; a.nz_cpu = c->nz_cpu; a.nz_mem = c->nz_mem;
  a.pod_count = c->pod_count; a.pods = c->pods; a.tcls = tcls; a.tclass = tclass; a.ncls = ncls; a.nb = nb; a.spec = spec;
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
