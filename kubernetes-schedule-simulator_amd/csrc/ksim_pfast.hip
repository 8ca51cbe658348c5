// ksim_pfast.hip — persistent-kernel mode specialised for resource-only pods (the C1/C3/C4/C5
// pod shape, ksim_is_fast_pod): used for a ksim_schedule() call whenever every pod of the call
// qualifies; ksim_persistent.hip handles everything else.
//
// Same protocol as ksim_persistent.hip — workgroup b keeps the name-rank range
// [b*chunk, (b+1)*chunk) in LDS, one control wave (wave 0) decides every pod redundantly from
// the tagged 8-byte granules all workgroups publish, seven row waves evaluate pod p+1 while
// the control wave decides pod p — with a shorter critical path:
//
//  * scores without a divide: each row keeps y = RN(1/alloc) (alloc is static).
//    LeastRequested / MostRequested floor(10x / cap) = trunc(x*y) corrected by the exact
//    remainder fma(-q, cap, x) (least_requested.go:44-53, most_requested.go:45-55);
//    BalancedResourceAllocation's float64(req)/float64(cap) (balanced_resource_allocation.go:
//    39-61) = Markstein's RN(a/b): q = a*y, r = fma(-q, b, a) (exact), RN(q + r*y) — the
//    correctly rounded quotient, bit-identical to the IEEE divide Go performs (y within half an
//    ulp of 1/b, q within one ulp of a/b, no over/underflow: operands are integers < 2^49).
//  * O(1) owner fix-up: the row waves keep the workgroup's top two (score, count) pairs of
//    pod p+1, so the owner of pod p's node removes that row's speculative evaluation and adds
//    its post-commit one with scalar arithmetic; the wave-level bitmasks it needs only if it
//    owns pod p+1 too are rebuilt after the correction is published.
//  * one prefix scan per decision: counts at the maximum give C (= its total) and the
//    workgroup holding the ix-th match from the top (core/generic_scheduler.go:183-198).
#include "ksim_fast.h"
#include "ksim_wave.h"

namespace {

constexpr int BS = 512;
constexpr int NW = BS / 64;     // waves per workgroup
constexpr int RW = NW - 1;      // row waves
constexpr int RT = RW * 64;     // row threads
constexpr int MAXB = 4;         // workgroups per sweep lane (grid <= 256)
constexpr int MAXG = 64 * MAXB;
constexpr int NSLOT = 4;        // granule slots (pod mod NSLOT)
constexpr int FIXSTRIDE = 16;   // fix granules 128 B apart
constexpr int RING = 16;        // pod-descriptor ring slots in LDS
constexpr int RING_FILL = 8;    // descriptors fetched per refill
constexpr uint64_t SPIN_LIMIT_TICKS = 200000000ull;  // s_memrealtime at 100 MHz = 2 s

typedef __attribute__((address_space(1))) uint64_t gu64;

__device__ __forceinline__ void store_granule(uint64_t* g, uint64_t v) {
  __hip_atomic_store((gu64*)g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t load_granule(const uint64_t* g) {
  return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// [slot][pos(b)], pos(b) = (b % MAXB) * 64 + b / MAXB: the sweep's j-th load of lane l is
// workgroup l*MAXB + j and each load instruction is 512 contiguous bytes.
__device__ __forceinline__ uint64_t* spec_at(uint64_t* gr, int slot, int b) {
  return gr + slot * MAXG + (b % MAXB) * 64 + b / MAXB;
}
__device__ __forceinline__ uint64_t* fix_at(uint64_t* gr, int slot) { return gr + NSLOT * MAXG + slot * FIXSTRIDE; }

// granule: tag:8 | fit:12 | count:12 | score:32 (-1 = no fit node)
__device__ __forceinline__ uint32_t gtag(uint64_t v) { return (uint32_t)(v >> 56); }
__device__ __forceinline__ int32_t gfit(uint64_t v) { return (int32_t)((v >> 44) & 0xFFF); }
__device__ __forceinline__ int32_t gcnt(uint64_t v) { return (int32_t)((v >> 32) & 0xFFF); }
__device__ __forceinline__ int32_t gscore(uint64_t v) { return (int32_t)(uint32_t)v; }
__device__ __forceinline__ uint64_t gpack(uint64_t tag, int32_t f, int32_t n, int32_t m) {
  return (tag << 56) | ((uint64_t)(uint32_t)f << 44) | ((uint64_t)(uint32_t)n << 32) | (uint64_t)(uint32_t)m;
}

#ifdef KSIM_STAMPS
#define STAMP(k)                                       \
  do {                                                 \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += t_ - t_prev;                         \
    t_prev = t_;                                      \
  } while (0)
#define OSTAMP(k)                                                          \
  do {                                                                     \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                     \
    if (lane == 0) atomicAdd((unsigned long long*)&c.dbg[k], t_ - o_prev); \
    o_prev = t_;                                                           \
  } while (0)
#else
#define STAMP(k) \
  do {           \
  } while (0)
#define OSTAMP(k) \
  do {            \
  } while (0)
#endif

struct FRow {
  int64_t ac, am, rc, rm, zc, zm;
  double dac, dam, yc, ym;  // alloc as float64 and RN(1/alloc) (0 when alloc == 0)
  int32_t allowed, count;
  uint32_t fl;
};

struct FRows {  // LDS image of the owned rows (SoA)
  int64_t *ac, *am, *rc, *rm, *zc, *zm;
  double *dac, *dam, *yc, *ym;
  int32_t *allowed, *count;
  uint32_t* fl;
  int32_t* ev;  // [2][chunk]: packed evaluation of pod p (parity p & 1), -1 = does not fit
};

constexpr int LDS_ROW_BYTES = 10 * 8 + 3 * 4 + 2 * 4;  // 100

extern __shared__ __attribute__((aligned(16))) char kf_smem[];

__device__ __forceinline__ FRows carve(int rows) {
  FRows r;
  int64_t* p = reinterpret_cast<int64_t*>(kf_smem);
  r.ac = p; r.am = p + rows; r.rc = p + 2 * rows; r.rm = p + 3 * rows; r.zc = p + 4 * rows; r.zm = p + 5 * rows;
  double* d = reinterpret_cast<double*>(p + 6 * rows);
  r.dac = d; r.dam = d + rows; r.yc = d + 2 * rows; r.ym = d + 3 * rows;
  int32_t* q = reinterpret_cast<int32_t*>(d + 4 * rows);
  r.allowed = q; r.count = q + rows;
  r.fl = reinterpret_cast<uint32_t*>(q + 2 * rows);
  r.ev = q + 3 * rows;
  return r;
}

__device__ __forceinline__ FRow load_frow(const FRows& R, int32_t j) {
  FRow r;
  r.ac = R.ac[j]; r.am = R.am[j]; r.rc = R.rc[j]; r.rm = R.rm[j]; r.zc = R.zc[j]; r.zm = R.zm[j];
  r.dac = R.dac[j]; r.dam = R.dam[j]; r.yc = R.yc[j]; r.ym = R.ym[j];
  r.allowed = R.allowed[j]; r.count = R.count[j]; r.fl = R.fl[j];
  return r;
}

// floor(x / b) for integers 0 <= x < 2^53, 0 < b < 2^49, y = RN(1/b): the estimate is off by
// at most one and the remainder fma(-q, b, x) is an exact integer.
__device__ __forceinline__ int32_t div_floor(double x, double b, double y) {
  double q = trunc(x * y);
  const double r = fma(-q, b, x);
  q = r < 0.0 ? q - 1.0 : (r >= b ? q + 1.0 : q);
  return (int32_t)q;
}
// RN(a / b) (Markstein): bit-identical to the IEEE divide.
__device__ __forceinline__ double quot(double a, double b, double y) {
  const double q = a * y;
  const double r = fma(-q, b, a);
  return fma(r, y, q);
}

// Weighted LeastRequested / MostRequested / BalancedResourceAllocation score of one node,
// tc/tm = pod non-zero request + node non-zero requested (resource_allocation.go:58-59).
__device__ __forceinline__ int64_t fscore(int64_t tc, int64_t tm, const FRow& r, int64_t wl, int64_t wm, int64_t wb) {
  if (((uint64_t)(tc | r.ac | tm | r.am)) >> 49) return ksim_slow_score(tc, r.ac, tm, r.am, wl, wm, wb);
  const bool okc = r.ac != 0 && tc <= r.ac, okm = r.am != 0 && tm <= r.am;
  int64_t s = 0;
  if (wl) {
    const int32_t lc = okc ? div_floor((double)(10 * (r.ac - tc)), r.dac, r.yc) : 0;
    const int32_t lm = okm ? div_floor((double)(10 * (r.am - tm)), r.dam, r.ym) : 0;
    s += wl * ((lc + lm) / 2);
  }
  if (wm) {
    const int32_t mc = okc ? div_floor((double)(10 * tc), r.dac, r.yc) : 0;
    const int32_t mm = okm ? div_floor((double)(10 * tm), r.dam, r.ym) : 0;
    s += wm * ((mc + mm) / 2);
  }
  if (wb) {
    const double fc = r.ac ? quot((double)tc, r.dac, r.yc) : 1.0;
    const double fm = r.am ? quot((double)tm, r.dam, r.ym) : 1.0;
    const int32_t b = (fc >= 1.0 || fm >= 1.0) ? 0 : (int32_t)((1.0 - fabs(fc - fm)) * 10.0);
    s += wb * b;
  }
  return s;
}

__device__ __forceinline__ int32_t feval(uint32_t preds, const KsimFastPod& P, const FRow& r, bool no_prio, int64_t wl,
                                         int64_t wm, int64_t wb, uint32_t& rm) {
  rm = ksim_fast_predicates(preds, P, r.ac, r.am, r.rc, r.rm, r.allowed, r.count, r.fl);
  const int32_t sc = no_prio ? 0 : (int32_t)fscore(P.nz_c + r.zc, P.nz_m + r.zm, r, wl, wm, wb);
  return rm ? -1 : sc;
}

// top-two (score, count) statistics of a set of packed evaluations
struct Top2 {
  int32_t f, m1, c1, m2, c2;
};
__device__ __forceinline__ void top2_add(Top2& t, int32_t m, int32_t n) {  // merge (m, n), n > 0, m >= 0
  if (m > t.m1) { t.m2 = t.m1; t.c2 = t.c1; t.m1 = m; t.c1 = n; }
  else if (m == t.m1) { t.c1 += n; }
  else if (m > t.m2) { t.m2 = m; t.c2 = n; }
  else if (m == t.m2) { t.c2 += n; }
}

}  // namespace

template <int NPT>
__global__ __launch_bounds__(BS) void ksim_pfast_kernel(KsimCtx c, uint64_t* granules) {
  __shared__ int32_t s_wst[2][RW][5];         // per row wave: fit, m1, c1, m2, c2 (by pod parity)
  __shared__ uint64_t s_fm[2][NPT][RW];       // per 64-row segment: fit rows
  __shared__ uint64_t s_bm[2][NPT][RW];       // ... rows at the wave maximum
  __shared__ int32_t s_wg[2][5];              // workgroup top-two of the pod
  __shared__ int32_t s_fix[2][2];             // {row the owner re-evaluated (-1 none), its reason mask}
  __shared__ int32_t s_hist[KSIM_NREASONS];
  __shared__ int32_t s_mode;
  __shared__ int32_t s_arr;
  __shared__ __attribute__((aligned(16))) ksim_pod s_pod[RING];
#ifdef KSIM_STAMPS
  uint64_t st_acc[16] = {};
#endif

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int rt = tid - 64;
  const int G = gridDim.x;
  const int me = blockIdx.x;
  const int64_t chunk = c.chunk;
  const int64_t lo = (int64_t)me * chunk;
  const int64_t hi = (lo + chunk < c.n) ? lo + chunk : c.n;
  const int32_t nrows = (int32_t)(hi - lo);
  const FRows R = carve((int)chunk);
  const uint32_t preds = c.preds;
  const int64_t wl = c.w[KSIM_W_LEAST_REQUESTED], wmr = c.w[KSIM_W_MOST_REQUESTED], wb = c.w[KSIM_W_BALANCED];
  const bool no_prio = c.no_prio != 0;

  for (int32_t j = tid; j < nrows; j += BS) {  // stage the owned rows into LDS
    const int64_t i = lo + j;
    const int64_t ac = c.alloc_cpu[i], am = c.alloc_mem[i];
    R.ac[j] = ac; R.am[j] = am;
    R.dac[j] = (double)ac; R.dam[j] = (double)am;
    R.yc[j] = ac ? 1.0 / (double)ac : 0.0;
    R.ym[j] = am ? 1.0 / (double)am : 0.0;
    R.rc[j] = c.req_cpu[i]; R.rm[j] = c.req_mem[i];
    R.zc[j] = c.nz_cpu[i]; R.zm[j] = c.nz_mem[i];
    R.allowed[j] = c.allowed_pods[i]; R.count[j] = c.pod_count[i]; R.fl[j] = c.flags[i];
  }
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
  uint64_t counter = *c.counter;  // replicated genericScheduler.lastNodeIndex
  __syncthreads();

  auto fpod = [&](int64_t p) -> KsimFastPod {
    const ksim_pod& P = s_pod[p % RING];
    return KsimFastPod{P.req_cpu, P.req_mem, P.nz_cpu, P.nz_mem, P.flags};
  };
  auto ptag = [&](int64_t p) -> uint64_t { return (uint64_t)((p - c.first + 1) & 0xFF); };
  // wave-level statistics of NPT entries per lane → LDS slot (buf, w)
  auto wave_stats = [&](const int32_t (&e)[NPT], int buf, int w) {
    int32_t v = -1, nf = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const uint64_t fm = __ballot(e[k] >= 0);
      nf += __popcll(fm);
      if (lane == 0) s_fm[buf][k][w - 1] = fm;
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
      const uint64_t bm = m1 < 0 ? 0ull : __ballot(e[k] == m1);
      c1 += __popcll(bm);
      c2 += m2 < 0 ? 0 : __popcll(__ballot(e[k] == m2));
      if (lane == 0) s_bm[buf][k][w - 1] = bm;
    }
    if (lane == 0) {
      s_wst[buf][w - 1][0] = nf; s_wst[buf][w - 1][1] = m1; s_wst[buf][w - 1][2] = c1;
      s_wst[buf][w - 1][3] = m2; s_wst[buf][w - 1][4] = c2;
    }
  };
  auto wg_top2 = [&](int buf) -> Top2 {
    Top2 t{0, -1, 0, -1, 0};
    int32_t s[RW][5];
#pragma unroll
    for (int w = 0; w < RW; ++w)
#pragma unroll
      for (int q = 0; q < 5; ++q) s[w][q] = s_wst[buf][w][q];
#pragma unroll
    for (int w = 0; w < RW; ++w) {
      t.f += s[w][0];
      if (s[w][2]) top2_add(t, s[w][1], s[w][2]);
      if (s[w][4]) top2_add(t, s[w][3], s[w][4]);
    }
    return t;
  };
  // row waves: the last one to finish pod p's statistics merges and publishes them
  auto arrive_publish = [&](int64_t p, int buf) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    int32_t old = 0;
    if (lane == 0) old = atomicAdd(&s_arr, 1);
    old = __builtin_amdgcn_readfirstlane(old);
    if ((old + 1) % RW == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      const Top2 t = wg_top2(buf);
      if (lane == 0) {
        s_wg[buf][0] = t.f; s_wg[buf][1] = t.m1; s_wg[buf][2] = t.c1; s_wg[buf][3] = t.m2; s_wg[buf][4] = t.c2;
        store_granule(spec_at(granules, (int)(p % NSLOT), me), gpack(ptag(p), t.f, t.c1, t.m1));
      }
    }
  };
  // row waves: evaluate pod p on every owned row
  auto eval_rows = [&](int64_t p, int32_t (&e)[NPT], uint32_t (&rm)[NPT], int32_t* ev) {
    const KsimFastPod F = fpod(p);
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int32_t j = k * RT + rt;
      e[k] = -1;
      rm[k] = 0;
      if (j < nrows) {
        e[k] = feval(preds, F, load_frow(R, j), no_prio, wl, wmr, wb, rm[k]);
        ev[j] = e[k];
      }
    }
  };

  // ---- prologue: statistics of the first pod ----
  uint32_t A_rm[NPT], B_rm[NPT];
  if (wv > 0) {
    int32_t e[NPT];
    eval_rows(c.first, e, A_rm, R.ev + (c.first & 1) * chunk);
    wave_stats(e, (int)(c.first & 1), wv);
    arrive_publish(c.first, (int)(c.first & 1));
  }
  int X = -1;  // control wave: owner workgroup of the previous pod's node (-1: none)
  __syncthreads();
#ifdef KSIM_STAMPS
  uint64_t t_prev = __builtin_amdgcn_s_memtime();
#endif

  for (int64_t pod = c.first; pod < c.end; ++pod) {
    const bool has_next = pod + 1 < c.end;
    const int pb = (int)(pod & 1);
    const int nb = (int)((pod + 1) & 1);
    int32_t jsel = -1;     // control wave: row committed by this workgroup
    int32_t e_new = -1;    // ... its evaluation of pod + 1 after the commit
    uint32_t rm_new = 0;
#ifdef KSIM_STAMPS
    uint64_t o_prev = 0;
#endif

    if (wv == 0) {
      // ---------------- a. sweep: every workgroup's granule of pod (+ the owner's fix) -------
      const uint64_t tag = ptag(pod);
      const int slot = (int)(pod % NSLOT);
      STAMP(1);
      uint64_t g[MAXB];
      bool ok = false;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
#pragma unroll
        for (int j = 0; j < MAXB; ++j) g[j] = load_granule(granules + slot * MAXG + j * 64 + lane);
        const uint64_t fx = load_granule(fix_at(granules, slot));
        bool mine = X < 0 || gtag(fx) == tag;
#pragma unroll
        for (int j = 0; j < MAXB; ++j) {
          const int b = lane * MAXB + j;
          mine &= (b >= G) || b == X || gtag(g[j]) == tag;
        }
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
      // ---------------- b. decide: findNodesThatFit count, max score, selectHost ------------
      int32_t f = 0, lm = -1;
#pragma unroll
      for (int j = 0; j < MAXB; ++j) {
        g[j] = (lane * MAXB + j < G) ? g[j] : 0;
        f += gfit(g[j]);
        lm = (gcnt(g[j]) && gscore(g[j]) > lm) ? gscore(g[j]) : lm;
      }
      const int32_t F = ksimw::sum_i32(f);
      const int32_t M0 = ksimw::max_i32(lm);
      int mode = 0, blk = -1, rank = 0;
      if (!ok) {
        mode = -1;
        if (lane == 0) atomicOr(c.err, 4);
      } else if (F == 1) {  // generic_scheduler.go:153-156: a single fit node skips selectHost
        mode = 1;
        int32_t jf = -1;
#pragma unroll
        for (int j = 0; j < MAXB; ++j) jf = gfit(g[j]) ? j : jf;
        const uint64_t hb = __ballot(jf >= 0);
        const int src = __builtin_ffsll((long long)hb) - 1;
        blk = src * MAXB + __builtin_amdgcn_readlane(jf, src);
      } else if (F > 1) {
        mode = 2;
        int32_t bm[MAXB], tot = 0;
#pragma unroll
        for (int j = 0; j < MAXB; ++j) {
          bm[j] = (gcnt(g[j]) && gscore(g[j]) == M0) ? gcnt(g[j]) : 0;
          tot += bm[j];
        }
        const int32_t pre = ksimw::prefix_incl_i32(tot);
        const uint32_t C = (uint32_t)__builtin_amdgcn_readlane(pre, 63);
        const int64_t ix = (counter >> 32) ? (int64_t)(counter % (uint64_t)C) : (int64_t)((uint32_t)counter % C);
        counter += 1;  // generic_scheduler.go:192-195
        const int64_t above = (int64_t)C - pre;  // matches in workgroups of higher lanes
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
      if (mode > 0 && blk == me) {
        // ---------------- c. owner: the rank-th row from the top, commit ----------------
        constexpr int S = NPT * RW;  // lane t = t-th 64-row segment from the top
        uint64_t m = 0;
        if (lane < S) {
          const int k = NPT - 1 - lane / RW, w = RW - 1 - lane % RW;
          m = (mode == 1) ? s_fm[pb][k][w] : (s_wst[pb][w][1] == M0 ? s_bm[pb][k][w] : 0ull);
        }
        const int32_t cnt = __popcll(m);
        const int32_t pre = ksimw::prefix_incl_i32(cnt);
        const uint64_t hm = __ballot(pre > rank);
        if (hm) {
          const int ts = __builtin_ffsll((long long)hm) - 1;
          const int32_t r2 = rank - (__builtin_amdgcn_readlane(pre, ts) - __builtin_amdgcn_readlane(cnt, ts));
          const uint64_t ms = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(m >> 32), ts) << 32) |
                              (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)m, ts);
          // the r2-th set bit counted from the top
          const bool is = ((ms >> lane) & 1ull) && __popcll((ms >> lane) >> 1) == r2;
          const uint64_t bb = __ballot(is);
          if (bb) {
            const int ks = NPT - 1 - ts / RW, ws = RW - 1 - ts % RW;
            jsel = ks * RT + ws * 64 + (__builtin_ffsll((long long)bb) - 1);
          }
        }
        OSTAMP(22);
        if (jsel < 0 || jsel >= nrows) {
          jsel = -1;
          mode = -1;
          if (lane == 0) atomicOr(c.err, 2);
        } else {
          const ksim_pod& P = s_pod[pod % RING];
          FRow r = load_frow(R, jsel);
          r.rc += P.add_cpu; r.rm += P.add_mem; r.zc += P.nz_cpu; r.zm += P.nz_mem; r.count += 1;
          if (lane == 0) {
            R.rc[jsel] = r.rc; R.rm[jsel] = r.rm; R.zc[jsel] = r.zc; R.zm[jsel] = r.zm; R.count[jsel] = r.count;
            c.out_node[pod] = (int32_t)(lo + jsel);
          }
          OSTAMP(23);
          if (has_next) e_new = feval(preds, fpod(pod + 1), r, no_prio, wl, wmr, wb, rm_new);
          OSTAMP(16);
        }
      }
      if (mode == 0 && me == 0 && lane == 0) c.out_node[pod] = -1;
      if (lane == 0) s_mode = mode;
      X = mode > 0 ? blk : -1;
      STAMP(6);
    } else {
      // ---------------- row waves: speculative evaluation of pod + 1 ----------------
      const bool refill = wv == 1 && ((pod - c.first) % RING_FILL) == 0;
      uint4 rv;
      if (refill) ring_load(pod + RING_FILL, rv);
#ifdef KSIM_STAMPS
      const uint64_t te0 = __builtin_amdgcn_s_memtime();
#endif
      if (has_next) {
        int32_t e[NPT];
        eval_rows(pod + 1, e, B_rm, R.ev + nb * chunk);
        wave_stats(e, nb, wv);
        arrive_publish(pod + 1, nb);
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

    if (wv == 0 && jsel >= 0 && has_next) {
      // ---------------- d. owner: correction of pod + 1's statistics, O(1) ----------------
      OSTAMP(17);
      const int32_t e_old = R.ev[nb * chunk + jsel];
      Top2 t{s_wg[nb][0], s_wg[nb][1], s_wg[nb][2], s_wg[nb][3], s_wg[nb][4]};
      if (e_old >= 0) {  // remove the speculative evaluation of the committed row
        t.f -= 1;
        if (e_old == t.m1) {
          if (--t.c1 == 0) { t.m1 = t.m2; t.c1 = t.c2; t.m2 = -1; t.c2 = 0; }
        } else if (e_old == t.m2) {
          if (--t.c2 == 0) { t.m2 = -1; }  // (a lower third value is not tracked: m2 is only
        }                                   //  consulted when the m1 row is removed, below)
      }
      int32_t F1 = t.f, M1 = t.m1, C1 = t.c1;
      if (e_new >= 0) {
        F1 += 1;
        if (e_new > M1) { M1 = e_new; C1 = 1; }
        else if (e_new == M1) { C1 += 1; }
      }
      if (C1 == 0) M1 = -1;
      if (lane == 0) store_granule(fix_at(granules, (int)((pod + 1) % NSLOT)), gpack(ptag(pod + 1), F1, C1, M1));
      OSTAMP(18);
      // off the critical path: the evaluation entry, the reasons and the wave's bitmasks
      const int w = 1 + (jsel % RT) / 64;
      int32_t e[NPT];
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int32_t j = k * RT + (w - 1) * 64 + lane;
        e[k] = (j == jsel) ? e_new : (j < nrows ? R.ev[nb * chunk + j] : -1);
      }
      wave_stats(e, nb, w);
      if (lane == 0) { R.ev[nb * chunk + jsel] = e_new; s_fix[nb][0] = jsel; s_fix[nb][1] = (int32_t)rm_new; }
      OSTAMP(19);
#ifdef KSIM_STAMPS
      if (lane == 0) atomicAdd((unsigned long long*)&c.dbg[21], 1ull);
#endif
    } else if (wv == 0 && lane == 0) {
      s_fix[nb][0] = -1;
    }

    if (mode == 0 && c.collect && c.out_reasons) {  // FitError: every workgroup adds its reasons
      if (tid < KSIM_NREASONS) s_hist[tid] = 0;
      __syncthreads();
      if (wv > 0) {
        const int32_t fr = s_fix[pb][0];
        const uint32_t fmk = (uint32_t)s_fix[pb][1];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const uint32_t rm = (k * RT + rt == fr) ? fmk : A_rm[k];
          for (int r = 0; r < KSIM_NREASONS; ++r) {
            const int32_t n = __popcll(__ballot((rm >> r) & 1u));
            if (lane == 0 && n) atomicAdd(&s_hist[r], n);
          }
        }
      }
      __syncthreads();
      if (tid < KSIM_NREASONS && s_hist[tid]) atomicAdd(&c.out_reasons[pod * KSIM_NREASONS + tid], s_hist[tid]);
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
    c.pod_count[i] = R.count[j];
  }
  if (me == 0 && tid == 0) {
    *c.counter = counter;
    *c.cursor = c.end;
  }
#ifdef KSIM_STAMPS
  if (me == 0 && tid == 0)
    for (int k = 0; k < 16; ++k) c.dbg[k] += (k == 5) ? 0 : st_acc[k];
  if (me == 0 && tid == 64) c.dbg[5] += st_acc[5];
#endif
}

// ---------------------------------------------------------------------------------------
static constexpr int PF_LDS_BUDGET = 150 * 1024;

// Same grid rule as ksim_persistent_config (one workgroup per CU, <= 256, >= 64 rows each).
extern "C" int ksim_pfast_config(int64_t n, int* grid, int* lds_rows) {
  int dev = 0;
  hipDeviceProp_t p;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return 0;
  int g = p.multiProcessorCount;
  if (g <= 0 || n <= 0) return 0;
  if (g > MAXG) g = MAXG;
  if (n < (int64_t)g * 64) g = (int)((n + 63) / 64);
  if (g < 1) g = 1;
  const int64_t chunk = (n + g - 1) / g;
  if (chunk * LDS_ROW_BYTES > PF_LDS_BUDGET || chunk > 4 * RT || chunk > 4095) return 0;
  *grid = g;
  *lds_rows = (int)chunk;
  return 1;
}

extern "C" size_t ksim_pfast_granule_bytes(void) { return (size_t)(NSLOT * MAXG + NSLOT * FIXSTRIDE) * sizeof(uint64_t); }

extern "C" hipError_t ksim_launch_pfast(const KsimCtx* c, uint64_t* granules, int grid, int lds_rows, hipStream_t s) {
  const size_t lds = (size_t)lds_rows * LDS_ROW_BYTES;
  if (lds_rows <= RT) hipLaunchKernelGGL((ksim_pfast_kernel<1>), dim3(grid), dim3(BS), lds, s, *c, granules);
  else if (lds_rows <= 2 * RT) hipLaunchKernelGGL((ksim_pfast_kernel<2>), dim3(grid), dim3(BS), lds, s, *c, granules);
  else hipLaunchKernelGGL((ksim_pfast_kernel<4>), dim3(grid), dim3(BS), lds, s, *c, granules);
  return hipGetLastError();
}
