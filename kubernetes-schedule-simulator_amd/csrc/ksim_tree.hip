// ksim_tree.hip — tree mode: the per-pod cycle of
// genericScheduler.Schedule (core/generic_scheduler.go:112-167) for resource-only pods under
// map-only policies, answered from incremental per-pod-class selection trees instead of an
// O(N) scan per pod.  Geometry and packing: ksim_tree.h.
//
// Why it is exact.  For a resource-only pod every predicate and every configured priority is a
// function of (pod class, node row) only (ksim_f64.h: kf64::feval), so a class's leaves are the
// per-node results findNodesThatFit + PrioritizeNodes would compute; the NormalizeReduce
// priorities have a single reduce class for such pods (host check), i.e. the same value on
// every fit node, and drop out of the argmax.  AddPod (node_info.go:318-341) changes one row,
// so after each commit only that node's leaf in every class, and the path above it, changes.
// Decision (per pod, from the class root): fit count 0 -> FitError (generic_scheduler.go:
// 136-141), 1 -> the only fit node without advancing lastNodeIndex (:147-150), else selectHost
// (:183-198): ix = lastNodeIndex % (count at max), lastNodeIndex++, and the ix-th max-score node
// in descending (score, name) order = the ix-th from the highest name rank, found by walking
// down the tree with a suffix count per level.
//
// One workgroup of 1024 threads (one CU) runs the whole pod range: wave 0 walks the tree for
// pod p (top levels in LDS, the rest in L2-resident HBM buffers), then all 16 waves commit: the
// row update and, for every class, the new leaf and the path to the root (the sibling groups of
// every level are loaded up front, one memory round trip).  No cross-CU traffic at all, so the
// per-pod cost is a few dependent L2 round trips, independent of N.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include "ksim_common.h"
#include "ksim_f64.h"
#include "ksim_tree.h"
#include "ksim_wave.h"

namespace {

constexpr int TB = KSIM_TREE_THREADS;
constexpr int TW = TB / 64;                                   // waves
constexpr int CW = TW - 1;                                    // waves 1..15 update the class paths
constexpr int CPW = (KSIM_TREE_MAX_CLASSES + CW - 1) / CW;    // classes per wave in the commit
constexpr int ML = KSIM_TREE_MAX_LEVELS;
constexpr int64_t LIM48 = (int64_t)1 << 48;
constexpr int64_t TREE_LDS_DEFAULT = 140 * 1024;

struct TreeArgs {
  KsimTreeGeo g;
  const int64_t* __restrict__ ac;
  const int64_t* __restrict__ am;
  int64_t* rc;
  int64_t* rm;
  int64_t* zc;
  int64_t* zm;
  const int32_t* __restrict__ allowed;
  int32_t* count;
  const uint32_t* __restrict__ fl;
  const ksim_pod* __restrict__ pods;
  const int32_t* __restrict__ tcls;
  const KsimTreeClass* __restrict__ cls;
  int32_t* leaves;
  uint64_t* levels;
  int32_t* fitc;  // [K] fit count per class
  int64_t first, end;
  uint64_t* counter;
  int64_t* cursor;
  int32_t* out_node;
  int32_t* out_reasons;
  int32_t* err;
  uint64_t* dbg;  // per-phase cycle sums (KSIM_STAMPS builds)
  kf64::EvCfg cfg;
  int32_t collect;
};

#ifdef KSIM_STAMPS
#define TSTAMP(k)                                      \
  do {                                                 \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    ts_acc[k] += t_ - ts_prev;                        \
    ts_prev = t_;                                     \
  } while (0)
#else
#define TSTAMP(k) \
  do {            \
  } while (0)
#endif

// Loads of data this launch writes: agent-scope relaxed atomics are never scalar loads and
// bypass the CU's vector L1, so after the writer's vmcnt(0) + barrier they read L2.
template <class T>
__device__ __forceinline__ T ldw(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every store of this wave has reached L2 (gfx9 counts stores in vmcnt)
__device__ __forceinline__ void stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Entry = (score + 1) << 32 | count at that score (0 = no fit node below).  Combining a wave's
// entries: DPP max of the high halves, then DPP sum of the counts at that maximum, both
// wave-uniform (ksimw patterns, total in lane 63).
__device__ __forceinline__ uint64_t wave_comb(uint32_t hi, uint32_t lo) {
  const int32_t H = ksimw::max_i32((int32_t)hi);
  const int32_t C = ksimw::sum_i32(hi == (uint32_t)H ? (int32_t)lo : 0);
  return ((uint64_t)(uint32_t)H << 32) | (uint32_t)C;
}
// a lane's M leaves -> (max score + 1, count at it); (0, 0) if none fits
template <int M>
__device__ __forceinline__ void lane_leaves(const int32_t* lv, uint32_t& hi, uint32_t& lo) {
  int32_t mx = -1;
#pragma unroll
  for (int t = 0; t < M; ++t) mx = max(mx, lv[t]);
  uint32_t c = 0;
#pragma unroll
  for (int t = 0; t < M; ++t) c += (lv[t] == mx) ? 1u : 0u;
  hi = (uint32_t)(mx + 1);
  lo = mx >= 0 ? c : 0u;
}

__device__ __forceinline__ kf64::FPod class_pod(const KsimTreeClass& c) {
  return kf64::FPod{c.rq_c, c.rq_m, c.nz_c, c.nz_m, 0.0, 0.0, c.anyreq, c.be};
}

__device__ __forceinline__ kf64::FRow load_row(const TreeArgs& a, int64_t i) {
  kf64::FRow r;
  r.ac = (double)a.ac[i];
  r.am = (double)a.am[i];
  r.yc = r.ac != 0.0 ? 1.0 / r.ac : 0.0;
  r.ym = r.am != 0.0 ? 1.0 / r.am : 0.0;
  r.rc = (double)ldw(a.rc + i);
  r.rm = (double)ldw(a.rm + i);
  r.zc = (double)ldw(a.zc + i);
  r.zm = (double)ldw(a.zm + i);
  r.allowed = a.allowed[i];
  r.count = ldw(a.count + i);
  r.fl = a.fl[i];
  return r;
}

// Lane holding the k-th match counted from the highest lane down (c = matches per lane);
// k becomes the rank inside that lane.  Returns -1 if the wave holds <= k matches.
__device__ __forceinline__ int pick_lane(uint32_t c, uint32_t& k) {
  const int32_t incl = ksimw::prefix_incl_i32((int32_t)c);
  const int32_t tot = __builtin_amdgcn_readlane(incl, 63);
  const uint32_t above = (uint32_t)(tot - incl);  // matches in higher lanes
  const uint64_t b = __ballot(above + c > k);
  if (b == 0) return -1;
  const int l = 63 - __clzll((long long)b);
  k -= (uint32_t)__builtin_amdgcn_readlane((int)above, l);
  return l;
}

// ---------------------------------------------------------------- tree build (per call if stale)
__global__ __launch_bounds__(256) void ksim_tree_leaf_kernel(TreeArgs a) {
  const int64_t st0 = a.g.st[0], tot = (int64_t)a.g.K * st0;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot; t += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(t / st0);
    const int64_t i = t - (int64_t)k * st0;
    int32_t v = -1;
    if (i < a.g.n) {
      uint32_t rmask;
      v = kf64::feval(a.cfg, class_pod(a.cls[k]), load_row(a, i), rmask);
    }
    a.leaves[t] = v;
  }
}

__global__ __launch_bounds__(256) void ksim_tree_level_kernel(TreeArgs a, int h) {
  const KsimTreeGeo& g = a.g;
  const int lane = threadIdx.x & 63;
  const int64_t sh = g.st[h], tot = (int64_t)g.K * sh;
  const int64_t wstep = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e < tot; e += wstep) {
    const int k = (int)(e / sh);
    const int64_t i = e - (int64_t)k * sh;
    uint64_t v = 0;
    if (i < g.nh[h]) {
      uint32_t hi = 0, lo = 0;
      if (h == 1) {
        const int32_t* L = a.leaves + (int64_t)k * g.st[0] + i * 64 * g.m + (int64_t)lane * g.m;
        int32_t mx = -1;
        for (int t = 0; t < g.m; ++t) mx = max(mx, L[t]);
        for (int t = 0; t < g.m; ++t) lo += (L[t] == mx) ? 1u : 0u;
        hi = (uint32_t)(mx + 1);
        if (mx < 0) lo = 0;
      } else {
        const uint64_t c = a.levels[g.goff[h - 1] + (int64_t)k * g.st[h - 1] + i * 64 + lane];
        hi = (uint32_t)(c >> 32);
        lo = (uint32_t)c;
      }
      v = wave_comb(hi, lo);
    }
    if (lane == 0) a.levels[g.goff[h] + e] = v;
  }
}

// fit count of every class (findNodesThatFit's len(filtered)); the tree kernel keeps it
// current with one add per class and commit
__global__ __launch_bounds__(256) void ksim_tree_fit_kernel(TreeArgs a) {
  __shared__ int32_t s_part[4];
  const int k = blockIdx.x;
  int32_t c = 0;
  for (int64_t i = threadIdx.x; i < a.g.n; i += 256) c += a.leaves[(int64_t)k * a.g.st[0] + i] >= 0;
  c = ksimw::sum_i32(c);
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) a.fitc[k] = s_part[0] + s_part[1] + s_part[2] + s_part[3];
}

// ---------------------------------------------------------------- the per-pod loop
extern __shared__ __attribute__((aligned(16))) uint64_t kt_lds[];  // levels hL..H

template <int M, int GL>
__global__ __launch_bounds__(TB) void ksim_tree_kernel(TreeArgs a) {
  __shared__ KsimTreeClass s_cls[KSIM_TREE_MAX_CLASSES];
  __shared__ int32_t s_fit[KSIM_TREE_MAX_CLASSES];   // fit count per class
  __shared__ int32_t s_vnew[KSIM_TREE_MAX_CLASSES];  // the committed node's new leaf per class
  __shared__ int32_t s_st[ML + 1], s_off[ML + 1];    // stride; offset (LDS for h >= hL, else global)
  __shared__ int32_t s_hist[KSIM_NREASONS];
  __shared__ int32_t s_sel, s_stop;
  __shared__ uint64_t s_chg;                         // classes whose leaf changed
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int K = a.g.K, H = a.g.H;
  constexpr int hL = GL + 1;  // levels 1..GL in global memory, hL..H in LDS
  constexpr int G0 = 64 * M;
  const int n = (int)a.g.n;
  const int gbase = (int)a.g.goff[hL];
  const int lds_entries = (int)a.g.lds_entries;
  for (int t = tid; t < lds_entries; t += TB) kt_lds[t] = a.levels[gbase + t];
  for (int t = tid; t < K; t += TB) {
    s_cls[t] = a.cls[t];
    s_fit[t] = a.fitc[t];
  }
  if (tid <= ML) {
    s_st[tid] = (int)a.g.st[tid];
    s_off[tid] = tid >= hL ? (int)(a.g.goff[tid] - gbase) : (int)a.g.goff[tid];
  }
  if (tid == 0) s_stop = 0;
  uint64_t counter = ldw(a.counter);
#ifdef KSIM_STAMPS
  uint64_t ts_acc[8] = {}, ts_prev = __builtin_amdgcn_s_memtime();
#endif
  __syncthreads();
  const int st0 = s_st[0];
  const uint64_t* root = kt_lds + s_off[H];  // st[H] == 1: one root per class
  int hist_cls = -1;
  int64_t p = a.first;
  int k_next = a.tcls[p];
  int64_t row_j = -1, row_c = 0, row_m = 0, row_zc = 0, row_zm = 0;  // thread 0: deferred row store
  int32_t row_n = 0;
  bool stop = false;
  while (p < a.end && !stop) {
    const int k = k_next;
    if (p + 1 < a.end) k_next = a.tcls[p + 1];
    const uint32_t F = (uint32_t)s_fit[k];
    if (F == 0) {  // FitError: no commit, lastNodeIndex unchanged
      if (tid == 0) a.out_node[p] = -1;
      if (a.collect) {
        if (hist_cls != k) {  // histogram of first-failing-predicate reasons over every node
          if (tid < KSIM_NREASONS) s_hist[tid] = 0;
          if (tid == 0 && row_j >= 0) {
            a.rc[row_j] = row_c; a.rm[row_j] = row_m; a.zc[row_j] = row_zc; a.zm[row_j] = row_zm; a.count[row_j] = row_n;
            row_j = -1;
          }
          stores_done();
          __syncthreads();
          const kf64::FPod P = class_pod(s_cls[k]);
          for (int i0 = 0; i0 < n; i0 += TB) {
            const int i = i0 + tid;
            uint32_t rm = 0;
            if (i < n) (void)kf64::feval(a.cfg, P, load_row(a, i), rm);
            if (__ballot(rm != 0))
              for (int r = 0; r < KSIM_NREASONS; ++r) {
                const int nr = __popcll(__ballot((rm >> r) & 1u));
                if (lane == 0 && nr) atomicAdd(&s_hist[r], nr);
              }
          }
          __syncthreads();
          hist_cls = k;
        }
        if (tid < KSIM_NREASONS) a.out_reasons[p * KSIM_NREASONS + tid] = s_hist[tid];
      }
      ++p;
      continue;
    }
    const uint64_t rt = root[k];
    const bool single = F == 1;
    uint32_t kth = 0;
    if (!single) {
      const uint32_t C = (uint32_t)rt;
      kth = (uint32_t)(counter % C);
      ++counter;
    }
    const uint32_t Sp = (uint32_t)(rt >> 32);  // maximum score + 1
    TSTAMP(0);
    if (wv == 0) {  // walk down: entry e of level h, kth match from the top
      int e = 0;
      bool bad = false;
      for (int h = H - 1; h >= 1; --h) {
        const int idx = s_off[h] + k * s_st[h] + e * 64 + lane;
        const uint64_t v = h >= hL ? kt_lds[idx] : ldw(a.levels + idx);
        const uint32_t vh = (uint32_t)(v >> 32);
        const uint32_t c = single ? (vh != 0u ? 1u : 0u) : (vh == Sp ? (uint32_t)v : 0u);
        const int l = pick_lane(c, kth);
        bad |= l < 0;
        e = e * 64 + (l < 0 ? 0 : l);
      }
      const int32_t* L = a.leaves + k * st0 + e * G0 + lane * M;
      int32_t lv[M];
#pragma unroll
      for (int t = 0; t < M; ++t) lv[t] = ldw(L + t);
      uint32_t c = 0;
#pragma unroll
      for (int t = 0; t < M; ++t) c += single ? (lv[t] >= 0) : ((uint32_t)(lv[t] + 1) == Sp);
      const int l = pick_lane(c, kth);
      bad |= l < 0;
      int sel = 0;
      uint32_t r = kth;
      bool found = false;
#pragma unroll
      for (int t = M - 1; t >= 0; --t) {
        const bool mt = single ? (lv[t] >= 0) : ((uint32_t)(lv[t] + 1) == Sp);
        if (mt && !found) {
          if (r == 0) { sel = t; found = true; } else { --r; }
        }
      }
      const int lsel = l < 0 ? 0 : l;
      const int node = e * G0 + lsel * M + __builtin_amdgcn_readlane(sel, lsel);
      if (lane == 0) {
        if (bad || node >= n) atomicOr(a.err, 16);  // tree inconsistent with its root
        s_sel = node < n ? node : 0;
        a.out_node[p] = node;
      }
    }
    TSTAMP(1);
    if (tid == 0 && row_j >= 0) {  // the previous pod's row (every wave has read it)
      a.rc[row_j] = row_c; a.rm[row_j] = row_m; a.zc[row_j] = row_zc; a.zm[row_j] = row_zm; a.count[row_j] = row_n;
    }
    stores_done();
    __syncthreads();
    TSTAMP(2);
    // ---- commit (Scheduler.assume -> NodeInfo.AddPod, node_info.go:318-341) ----
    const int j = s_sel;
    const int e1 = j / G0;
    const int lj = (j - e1 * G0) / M, sj = j % M;
    // leaf groups and global-level sibling groups of this wave's classes (waves 1..15), issued
    // now so they arrive while wave 0 evaluates the new row
    int32_t lv[CPW][M];
    uint64_t gsib[CPW][GL > 0 ? GL : 1];
#pragma unroll
    for (int q = 0; q < CPW; ++q) {
      const int kc = wv - 1 + q * CW;
      if (wv > 0 && kc < K) {
        const int32_t* L = a.leaves + kc * st0 + e1 * G0 + lane * M;
#pragma unroll
        for (int t = 0; t < M; ++t) lv[q][t] = ldw(L + t);
        int e = e1;
#pragma unroll
        for (int h = 1; h <= GL; ++h) {
          gsib[q][h - 1] = ldw(a.levels + s_off[h] + kc * s_st[h] + (e >> 6) * 64 + lane);
          e >>= 6;
        }
      }
    }
    if (wv == 0) {  // the new row and every class's new leaf (lane c = class c)
      const ksim_pod& P = a.pods[p];
      const int64_t nrc = ldw(a.rc + j) + P.add_cpu, nrm = ldw(a.rm + j) + P.add_mem;
      const int64_t nzc = ldw(a.zc + j) + P.nz_cpu, nzm = ldw(a.zm + j) + P.nz_mem;
      const int32_t ncnt = ldw(a.count + j) + 1;
      const int32_t vold = lane < K ? ldw(a.leaves + lane * st0 + j) : -1;
      kf64::FRow nr;
      nr.ac = (double)a.ac[j];
      nr.am = (double)a.am[j];
      nr.yc = nr.ac != 0.0 ? 1.0 / nr.ac : 0.0;
      nr.ym = nr.am != 0.0 ? 1.0 / nr.am : 0.0;
      nr.rc = (double)nrc; nr.rm = (double)nrm; nr.zc = (double)nzc; nr.zm = (double)nzm;
      nr.allowed = a.allowed[j];
      nr.count = ncnt;
      nr.fl = a.fl[j];
      uint32_t rmask;
      const int32_t vnew = kf64::feval(a.cfg, class_pod(s_cls[lane < K ? lane : 0]), nr, rmask);
      const bool chg = lane < K && vnew != vold;
      const uint64_t cm = __ballot(chg);
      if (lane < K) {
        s_vnew[lane] = vnew;
        s_fit[lane] += (vnew >= 0 ? 1 : 0) - (vold >= 0 ? 1 : 0);
      }
      if (chg) a.leaves[lane * st0 + j] = vnew;
      if (lane == 0) {
        s_chg = cm;
        // quantities must stay exact in float64 (ksim_f64.h): stop after this pod otherwise
        s_stop = nrc >= LIM48 || nrm >= LIM48 || nzc >= LIM48 || nzm >= LIM48;
        row_j = j; row_c = nrc; row_m = nrm; row_zc = nzc; row_zm = nzm; row_n = ncnt;
      }
    }
    __syncthreads();
    TSTAMP(3);
    const uint64_t chg = s_chg;
#pragma unroll
    for (int q = 0; q < CPW; ++q) {
      const int kc = wv - 1 + q * CW;
      if (wv > 0 && kc < K && ((chg >> kc) & 1ull)) {  // the path from leaf j up, until an entry is unchanged
        const int32_t v = s_vnew[kc];
        if (lane == lj) {
#pragma unroll
          for (int t = 0; t < M; ++t)
            if (t == sj) lv[q][t] = v;
        }
        uint32_t hi, lo;
        lane_leaves<M>(lv[q], hi, lo);
        uint64_t acc = wave_comb(hi, lo);
        int e = e1;
        bool done = false;
#pragma unroll
        for (int h = 1; h <= GL; ++h) {  // global levels (h < hL <= H)
          if (!done) {
            const int sl = e & 63;
            const uint64_t old = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(gsib[q][h - 1] >> 32), sl) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)gsib[q][h - 1], sl);
            if (old == acc) {
              done = true;
            } else {
              if (lane == 0) a.levels[s_off[h] + kc * s_st[h] + e] = acc;
              const uint64_t x = lane == sl ? acc : gsib[q][h - 1];
              acc = wave_comb((uint32_t)(x >> 32), (uint32_t)x);
              e >>= 6;
            }
          }
        }
        if (!done) {
          for (int h = hL; h <= H; ++h) {  // LDS levels
            const int base = s_off[h] + kc * s_st[h];
            if (kt_lds[base + e] == acc) break;
            if (lane == 0) kt_lds[base + e] = acc;
            if (h == H) break;
            const uint64_t x = lane == (e & 63) ? acc : kt_lds[base + (e >> 6) * 64 + lane];
            acc = wave_comb((uint32_t)(x >> 32), (uint32_t)x);
            e >>= 6;
          }
        }
      }
    }
    TSTAMP(4);
    hist_cls = -1;
    stop = s_stop != 0;
    ++p;
    stores_done();
    __syncthreads();
    TSTAMP(5);
  }
  if (tid == 0 && row_j >= 0) {
    a.rc[row_j] = row_c; a.rm[row_j] = row_m; a.zc[row_j] = row_zc; a.zm[row_j] = row_zm; a.count[row_j] = row_n;
  }
  stores_done();
  __syncthreads();
  for (int t = tid; t < lds_entries; t += TB) a.levels[gbase + t] = kt_lds[t];
  for (int t = tid; t < K; t += TB) a.fitc[t] = s_fit[t];
  if (tid == 0) {
    __hip_atomic_store(a.counter, counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.cursor, p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (stop) atomicOr(a.err, 8);
#ifdef KSIM_STAMPS
    for (int k = 0; k < 6; ++k) atomicAdd((unsigned long long*)&a.dbg[k], (unsigned long long)ts_acc[k]);
    atomicAdd((unsigned long long*)&a.dbg[8], (unsigned long long)(p - a.first));
#endif
  }
}

TreeArgs make_args(const KsimCtx* c, const KsimTreeGeo* g, const KsimTreeClass* cls, const int32_t* tcls,
                   int32_t* leaves, uint64_t* levels, int32_t* fitc) {
  TreeArgs a{};
  a.g = *g;
  a.ac = c->alloc_cpu; a.am = c->alloc_mem;
  a.rc = c->req_cpu; a.rm = c->req_mem; a.zc = c->nz_cpu; a.zm = c->nz_mem;
  a.allowed = c->allowed_pods; a.count = c->pod_count; a.fl = c->flags;
  a.pods = c->pods; a.tcls = tcls; a.cls = cls;
  a.leaves = leaves; a.levels = levels; a.fitc = fitc;
  a.first = c->first; a.end = c->end;
  a.counter = c->counter; a.cursor = c->cursor; a.out_node = c->out_node; a.out_reasons = c->out_reasons;
  a.err = c->err;
  a.dbg = c->dbg;
  a.cfg = kf64::make_evcfg(c->preds, c->no_prio != 0, (int32_t)c->w[KSIM_W_LEAST_REQUESTED],
                           (int32_t)c->w[KSIM_W_MOST_REQUESTED], (int32_t)c->w[KSIM_W_BALANCED]);
  a.collect = c->collect;
  return a;
}

}  // namespace

extern "C" int ksim_tree_plan(int64_t n, int32_t K, int64_t budget, int32_t force_m, KsimTreeGeo* out) {
  if (n <= 0 || n >= ((int64_t)1 << 24) || K <= 0 || K > KSIM_TREE_MAX_CLASSES || !out) return 0;
  if (budget <= 0) budget = TREE_LDS_DEFAULT;
  bool found = false;
  int64_t best = INT64_MAX;
  for (int m : {1, 2, 4}) {
    if (force_m && m != force_m) continue;
    KsimTreeGeo g{};
    g.n = n; g.K = K; g.m = m;
    const int64_t G0 = 64 * m;
    g.nh[0] = n;
    g.nh[1] = (n + G0 - 1) / G0;
    int H = 1;
    while (g.nh[H] > 1 && H < KSIM_TREE_MAX_LEVELS) { g.nh[H + 1] = (g.nh[H] + 63) / 64; ++H; }
    if (g.nh[H] > 1) continue;
    g.H = H;
    g.st[0] = g.nh[1] * G0;
    for (int h = 1; h <= H; ++h) g.st[h] = h == H ? 1 : g.nh[h + 1] * 64;
    int hL = H + 1;
    int64_t bytes = 0;
    for (int h = H; h >= 1; --h) {
      const int64_t b = bytes + (int64_t)K * g.st[h] * 8;
      if (b > budget) break;
      bytes = b;
      hL = h;
    }
    if (hL > H || hL - 1 > (m == 4 ? 0 : m == 2 ? 1 : 2)) continue;  // the instantiated <M, GL> forms (no scratch)
    if ((int64_t)K * g.st[0] >= INT32_MAX) continue;  // 32-bit indices in the kernel
    g.hL = hL;
    g.goff[1] = 0;
    for (int h = 1; h < H; ++h) g.goff[h + 1] = g.goff[h] + (int64_t)K * g.st[h];
    g.level_entries = g.goff[H] + (int64_t)K * g.st[H];
    for (int h = 0; h <= KSIM_TREE_MAX_LEVELS; ++h) g.loff[h] = h >= hL && h <= H ? (int32_t)(g.goff[h] - g.goff[hL]) : -1;
    g.lds_entries = bytes / 8;
    // dependent global round trips of the walk (leaf level + levels below hL) dominate; then
    // the bytes every commit loads
    const int64_t cost = (int64_t)hL * 1000 + (int64_t)K * (G0 * 4 + (hL - 1) * 512) / 64;
    if (cost < best) { best = cost; *out = g; found = true; }
  }
  return found ? 1 : 0;
}

extern "C" hipError_t ksim_tree_build(const KsimCtx* c, const KsimTreeGeo* g, const KsimTreeClass* cls,
                                      const int32_t* tcls, int32_t* leaves, uint64_t* levels, int32_t* fitc,
                                      hipStream_t s) {
  const TreeArgs a = make_args(c, g, cls, tcls, leaves, levels, fitc);
  const int64_t tl = (int64_t)g->K * g->st[0];
  hipLaunchKernelGGL(ksim_tree_leaf_kernel, dim3((unsigned)std::min<int64_t>((tl + 255) / 256, 8192)), dim3(256), 0, s, a);
  for (int h = 1; h <= g->H; ++h) {
    const int64_t waves = (int64_t)g->K * g->st[h];
    hipLaunchKernelGGL(ksim_tree_level_kernel, dim3((unsigned)std::min<int64_t>((waves + 3) / 4, 8192)), dim3(256), 0, s, a, h);
  }
  hipLaunchKernelGGL(ksim_tree_fit_kernel, dim3(g->K), dim3(256), 0, s, a);
  return hipGetLastError();
}

extern "C" hipError_t ksim_tree_launch(const KsimCtx* c, const KsimTreeGeo* g, const KsimTreeClass* cls,
                                       const int32_t* tcls, int32_t* leaves, uint64_t* levels, int32_t* fitc,
                                       hipStream_t s) {
  const TreeArgs a = make_args(c, g, cls, tcls, leaves, levels, fitc);
  const size_t lds = (size_t)g->lds_entries * sizeof(uint64_t);
#define KT_CASE(MM, GG) \
  if (g->m == MM && g->hL == GG + 1) { hipLaunchKernelGGL((ksim_tree_kernel<MM, GG>), dim3(1), dim3(TB), lds, s, a); return hipGetLastError(); }
  KT_CASE(1, 0) KT_CASE(1, 1) KT_CASE(1, 2) KT_CASE(2, 0) KT_CASE(2, 1) KT_CASE(4, 0)
#undef KT_CASE
  return hipErrorInvalidValue;
}
