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
// One wave on one CU runs the whole pod range with no barrier per pod: it walks the tree for
// pod p (top levels in LDS, the rest in L2/MALL-resident HBM buffers), commits the row,
// evaluates the committed node for every class at once (lane c = class c), and updates each
// changed class's leaf-to-root path lane-parallel with an O(1) parent rule, re-combining a
// sibling group only where a unique maximum dropped.  A second wave streams pod descriptors
// into an LDS ring ahead of it.  No cross-CU traffic at all: the per-pod cost is a few
// dependent L2/MALL round trips plus one vector evaluation, independent of N.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include "ksim_common.h"
#include "ksim_f64.h"
#include "ksim_tree.h"
#include "ksim_wave.h"

namespace {

#ifndef KSIM_TREE_VAR
#define KSIM_TREE_VAR 0  // diagnostic variants of the stamps build (tools/gpu_tree_ab.sh)
#endif
constexpr int ML = KSIM_TREE_MAX_LEVELS;
constexpr int LS = 2;  // LDS levels below the root (plan limit)
constexpr int64_t LIM48 = (int64_t)1 << 48;
constexpr int64_t TREE_LDS_DEFAULT = 148 * 1024;  // + ~8.6 KB static LDS (classes, pod ring) < 160 KB

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
  double* ty;     // [2][n] RN(1/alloc cpu), RN(1/alloc mem) (0 for a zero allocatable)
  int64_t first, end;
  uint64_t* counter;
  int64_t* cursor;
  int32_t* out_node;
  int32_t* out_reasons;
  int32_t* err;
  uint64_t* dbg;  // per-phase cycle sums (KSIM_STAMPS builds)
  kf64::EvCfg cfg;
  int32_t collect;
  // scenario sweep (ksim_sweep): nsc > 0 independent copies of the cluster, block / slice s =
  // scenario s with its own dynamic columns, trees, counter, weights and output row
  int32_t nsc;
  const kf64::EvCfg* sw_cfg;
  int64_t sw_count;  // output row length (pods of the call)
};

// Scenario s's view of the arguments (nsc > 0).
__device__ __forceinline__ void scen_ptrs(TreeArgs& a, int s) {
  const int64_t n = a.g.n;
  a.rc += s * n; a.rm += s * n; a.zc += s * n; a.zm += s * n; a.count += s * n;
  a.leaves += (int64_t)s * a.g.K * a.g.st[0];
  a.levels += (int64_t)s * a.g.level_entries;
  a.fitc += (int64_t)s * a.g.K;
  a.counter += s;
  a.out_node += (int64_t)s * a.sw_count - a.first;
  a.cfg = a.sw_cfg[s];
}

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
// a lane's M consecutive leaves in one load (nontemporal: served by L2, like ldw)
typedef int32_t v2i __attribute__((ext_vector_type(2)));
typedef int32_t v4i __attribute__((ext_vector_type(4)));
template <int M>
__device__ __forceinline__ void ld_leaves(const int32_t* L, int32_t* lv) {
  if constexpr (M == 4) {
#if KSIM_TREE_VAR == 1
    const v4i x = *(const volatile v4i*)L;
#else
    const v4i x = __builtin_nontemporal_load((const v4i*)L);
#endif
    lv[0] = x.x; lv[1] = x.y; lv[2] = x.z; lv[3] = x.w;
  } else if constexpr (M == 2) {
    const v2i x = __builtin_nontemporal_load((const v2i*)L);
    lv[0] = x.x; lv[1] = x.y;
  } else {
    lv[0] = ldw(L);
  }
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

constexpr int RING = 128;
// x % c for selectHost's ix (c < 2^24): a float64 quotient corrected by the exact remainder
// below 2^52, the 64-bit divide beyond
__device__ __forceinline__ uint32_t mod_u64(uint64_t x, uint32_t c) {
  if (x < (1ull << 52)) {
    const double q = trunc((double)x / (double)c);
    int64_t r = (int64_t)x - (int64_t)q * (int64_t)c;
    if (r < 0) r += c;
    else if (r >= (int64_t)c) r -= c;
    return (uint32_t)r;
  }
  return (uint32_t)(x % c);
}

// ---------------------------------------------------------------- tree build (per call if stale)
__global__ __launch_bounds__(256) void ksim_tree_leaf_kernel(TreeArgs a0) {
  const int64_t st0 = a0.g.st[0], per = (int64_t)a0.g.K * st0, tot = per * max(1, a0.nsc);
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot; t += (int64_t)gridDim.x * blockDim.x) {
    const int sc = (int)(t / per);
    const int64_t r = t - sc * per;
    const int k = (int)(r / st0);
    const int64_t i = r - (int64_t)k * st0;
    TreeArgs a = a0;
    if (a0.nsc) scen_ptrs(a, sc);
    int32_t v = -1;
    if (i < a.g.n) {
      uint32_t rmask;
      v = kf64::feval(a.cfg, class_pod(a.cls[k]), load_row(a, i), rmask);
    }
    a.leaves[r] = v;
    if (sc == 0 && k == 0 && i < a.g.n) {
      a.ty[i] = a.ac[i] ? 1.0 / (double)a.ac[i] : 0.0;
      a.ty[a.g.n + i] = a.am[i] ? 1.0 / (double)a.am[i] : 0.0;
    }
  }
}

__global__ __launch_bounds__(256) void ksim_tree_level_kernel(TreeArgs a0, int h) {
  const KsimTreeGeo& g = a0.g;
  const int lane = threadIdx.x & 63;
  const int64_t sh = g.st[h], per = (int64_t)g.K * sh, tot = per * max(1, a0.nsc);
  const int64_t wstep = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t e0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e0 < tot; e0 += wstep) {
    const int sc = (int)(e0 / per);
    const int64_t e = e0 - sc * per;
    TreeArgs a = a0;
    if (a0.nsc) scen_ptrs(a, sc);
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
__global__ __launch_bounds__(256) void ksim_tree_fit_kernel(TreeArgs a0) {
  __shared__ int32_t s_part[4];
  TreeArgs a = a0;
  if (a0.nsc) scen_ptrs(a, blockIdx.x / a0.g.K);
  const int k = blockIdx.x % a0.g.K;
  int32_t c = 0;
  for (int64_t i = threadIdx.x; i < a.g.n; i += 256) c += a.leaves[(int64_t)k * a.g.st[0] + i] >= 0;
  c = ksimw::sum_i32(c);
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) a.fitc[k] = s_part[0] + s_part[1] + s_part[2] + s_part[3];
}

// ---------------------------------------------------------------- the per-pod loop
extern __shared__ __attribute__((aligned(16))) uint64_t kt_lds[];  // levels hL..H

// O(1) update of a parent entry P when one child's entry goes from co to cn (entries are
// (max + 1) << 32 | count at max): false if the parent's maximum vanished from this child and
// the siblings must be re-combined.
__device__ __forceinline__ bool parent_rule(uint64_t P, uint64_t co, uint64_t cn, uint64_t& NP) {
  const uint32_t ph = (uint32_t)(P >> 32), pc = (uint32_t)P;
  const uint32_t oh = (uint32_t)(co >> 32), nh = (uint32_t)(cn >> 32);
  if (nh > ph) { NP = cn; return true; }
  const int64_t c = (int64_t)pc - (oh == ph ? (int64_t)(uint32_t)co : 0) + (nh == ph ? (int64_t)(uint32_t)cn : 0);
  if (c > 0 || ph == 0) { NP = ((uint64_t)ph << 32) | (uint32_t)c; return true; }
  return false;
}
__device__ __forceinline__ uint64_t leaf_entry(int32_t v) { return v < 0 ? 0ull : ((uint64_t)(v + 1) << 32) | 1u; }

// Wave-cooperative re-combination of entry eh of level h for class c from its children (all
// already updated this pod).
template <int M, int GL>
__device__ __forceinline__ uint64_t rescan(const TreeArgs& a, const int32_t* s_st, const int32_t* s_off, int c, int h,
                                           int eh, int lane) {
  constexpr int hL = GL + 1;
  if (h == 1) {
    int32_t lv[M];
    ld_leaves<M>(a.leaves + c * s_st[0] + eh * 64 * M + lane * M, lv);
    uint32_t hi, lo;
    lane_leaves<M>(lv, hi, lo);
    return wave_comb(hi, lo);
  }
  const int idx = s_off[h - 1] + c * s_st[h - 1] + eh * 64 + lane;
  const uint64_t x = h - 1 >= hL ? kt_lds[idx] : ldw(a.levels + idx);
  return wave_comb((uint32_t)(x >> 32), (uint32_t)x);
}

// One workgroup of two waves on one CU.  Wave 0 schedules every pod alone — no barrier on the
// per-pod path: decide from the class root (LDS), walk down (LDS levels, then global levels and
// the leaf group), commit the row, evaluate the committed node for every class (lane c = class
// c), and update each changed class's path lane-parallel with the O(1) parent rule, re-combining
// a sibling group (wave-cooperative) only where a unique maximum dropped.  Wave 1 streams pod
// descriptors into an LDS ring ahead of wave 0.
template <int M, int GL>
__global__ __launch_bounds__(128) void ksim_tree_kernel(TreeArgs a0) {
  TreeArgs a = a0;
  if (a0.nsc) scen_ptrs(a, blockIdx.x);
  __shared__ KsimTreeClass s_cls[KSIM_TREE_MAX_CLASSES];
  __shared__ int32_t s_fit[KSIM_TREE_MAX_CLASSES];   // fit count per class
  __shared__ int32_t s_st[ML + 1], s_off[ML + 1];    // stride; offset (LDS for h >= hL, else global)
  __shared__ int32_t s_hist[KSIM_NREASONS];
  __shared__ int32_t s_rk[RING];                     // pod ring: tree class
  __shared__ int64_t s_rd[4][RING];                  // pod ring: add_cpu, add_mem, nz_cpu, nz_mem
  __shared__ int64_t s_rtag[RING];                   // pod ring: the pod a slot holds
  __shared__ int64_t s_done;                         // pods wave 0 has finished
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int K = a.g.K, H = a.g.H;
  constexpr int hL = GL + 1;  // levels 1..GL in global memory, hL..H in LDS
  constexpr int G0 = 64 * M;
  const int n = (int)a.g.n;
  const int gbase = (int)a.g.goff[hL];
  const int lds_entries = (int)a.g.lds_entries;
  for (int t = tid; t < lds_entries; t += 128) kt_lds[t] = a.levels[gbase + t];
  for (int t = tid; t < K; t += 128) {
    s_cls[t] = a.cls[t];
    s_fit[t] = a.fitc[t];
  }
  if (tid <= ML) {
    s_st[tid] = (int)a0.g.st[tid];
    s_off[tid] = tid >= hL ? (int)(a0.g.goff[tid] - gbase) : (int)a0.g.goff[tid];
  }
  for (int t = tid; t < RING; t += 128) s_rtag[t] = -1;
  if (tid == 0) s_done = a.first;
  __syncthreads();

  if (wv == 1) {  // ---- pod ring producer: 64 pods at a time, at most RING ahead of wave 0
    for (int64_t q0 = a.first; q0 < a.end; q0 += 64) {
      uint32_t spins = 0;
      int64_t done;
      while ((done = __hip_atomic_load(&s_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < q0 + 64 - RING) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1u << 28)) { if (lane == 0) atomicOr(a.err, 32); return; }
      }
      if (done == INT64_MAX) return;  // wave 0 stopped early
      const int64_t q = q0 + lane;
      if (q < a.end) {
        const int r = (int)(q & (RING - 1));
        const ksim_pod& P = a.pods[q];
        s_rk[r] = a.tcls[q];
        s_rd[0][r] = P.add_cpu; s_rd[1][r] = P.add_mem; s_rd[2][r] = P.nz_cpu; s_rd[3][r] = P.nz_mem;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");  // LDS only: no wait on global stores
        __hip_atomic_store(&s_rtag[r], q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    return;
  }

  // ---- wave 0: the scheduler
  const int st0 = s_st[0];
  const uint64_t* root = kt_lds + s_off[H];  // st[H] == 1: one root per class
  // lastNodeIndex in scalar registers: loaded (and waited for) once, not a vector register whose
  // pending load makes every pod wait for all of the previous pod's stores
  uint64_t counter;
  {
    const uint64_t c0 = ldw(a.counter);
    counter = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(c0 >> 32)) << 32) |
              (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)c0);
  }
#ifdef KSIM_STAMPS
  uint64_t ts_acc[8] = {}, ts_prev = __builtin_amdgcn_s_memtime();
#endif
  // per-class root entry and fit count in registers, lane c = class c (K <= 64): the decision
  // reads them with readlane instead of two dependent LDS loads; LDS keeps the root level too
  uint64_t rootv = lane < K ? root[lane] : 0ull;
  int32_t fitv = lane < K ? s_fit[lane] : 0;
  // lane k: the last pod of class k whose FitError histogram (in out_reasons) still holds — a
  // failing pod commits nothing, so until the next commit every class's histogram stays valid
  // (past saturation, where nearly every pod fails, each class is scanned once per commit)
  int64_t hist_pod = -1;
  int64_t p = a.first;
  int64_t ready = a.first;  // pods below this are in the ring
  bool stop = false;
  while (p < a.end && !stop) {
    const int rs = (int)(p & (RING - 1));
    if (p >= ready) {  // once per producer batch: its last pod's tag (the producer's release fence
                       // orders every lane's slot writes before any of the batch's tags)
      const int64_t ql = min(a.first + ((p - a.first) & ~(int64_t)63) + 63, a.end - 1);
      ready = ql + 1;
      uint32_t spins = 0;
      while (__hip_atomic_load(&s_rtag[ql & (RING - 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != ql) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 28)) { if (lane == 0) atomicOr(a.err, 32); stop = true; break; }
      }
      if (stop) break;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    }
    const int k = __builtin_amdgcn_readfirstlane(s_rk[rs]);
    const int64_t pc = s_rd[0][rs], pm = s_rd[1][rs], pzc = s_rd[2][rs], pzm = s_rd[3][rs];  // commit deltas
    const uint32_t F = (uint32_t)__builtin_amdgcn_readlane(fitv, k);
    if (F == 0) {  // FitError: no commit, lastNodeIndex unchanged
      if (lane == 0) a.out_node[p] = -1;
      if (a.collect) {
        const int64_t pk = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)((uint64_t)hist_pod >> 32), k) << 32) |
                                     (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)hist_pod, k));
        if (pk >= 0) {  // same wave wrote it: program order makes the load see the store
          if (lane < KSIM_NREASONS) a.out_reasons[p * KSIM_NREASONS + lane] = a.out_reasons[pk * KSIM_NREASONS + lane];
        } else {  // histogram of first-failing-predicate reasons over every node
          if (lane < KSIM_NREASONS) s_hist[lane] = 0;
          const kf64::FPod P = class_pod(s_cls[k]);
          for (int i0 = 0; i0 < n; i0 += 64) {
            const int i = i0 + lane;
            uint32_t rm = 0;
            if (i < n) (void)kf64::feval(a.cfg, P, load_row(a, i), rm);
            if (__ballot(rm != 0))
              for (int r = 0; r < KSIM_NREASONS; ++r) {
                const int nr = __popcll(__ballot((rm >> r) & 1u));
                if (lane == 0 && nr) s_hist[r] += nr;
              }
          }
          hist_pod = lane == k ? p : hist_pod;
          if (lane < KSIM_NREASONS) a.out_reasons[p * KSIM_NREASONS + lane] = s_hist[lane];
        }
      }
      ++p;
      if (lane == 0) __hip_atomic_store(&s_done, p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      continue;
    }
    const uint64_t rt = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(rootv >> 32), k) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)rootv, k);
    const bool single = F == 1;
    uint32_t kth = 0;
    if (!single) {
      kth = mod_u64(counter, (uint32_t)rt);
      ++counter;
    }
    const uint32_t Sp = (uint32_t)(rt >> 32);  // maximum score + 1
    TSTAMP(0);
    // ---- walk down: entry e of level h, kth match from the top ----
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
    int j;
    {
      TSTAMP(4);
      int32_t lv[M];
      ld_leaves<M>(a.leaves + k * st0 + e * G0 + lane * M, lv);
      uint32_t c = 0;
#pragma unroll
      for (int t = 0; t < M; ++t) c += single ? (lv[t] >= 0) : ((uint32_t)(lv[t] + 1) == Sp);
#ifdef KSIM_STAMPS
      asm volatile("" ::"v"(c));  // the leaf values are in
#endif
      TSTAMP(5);
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
      j = e * G0 + lsel * M + __builtin_amdgcn_readlane(sel, lsel);
      if (bad || j >= n) {  // tree inconsistent with its root
        if (lane == 0) atomicOr(a.err, 16);
        j = 0;
      }
    }
    TSTAMP(1);
    // ---- commit (Scheduler.assume -> NodeInfo.AddPod, node_info.go:318-341) ----
    const int e1 = j / G0;
    const bool cl = lane < K;
    const int cc = cl ? lane : 0;  // lane c = class c
    const int64_t nrc = ldw(a.rc + j) + pc, nrm = ldw(a.rm + j) + pm;
    const int64_t nzc = ldw(a.zc + j) + pzc, nzm = ldw(a.zm + j) + pzm;
    const int32_t ncnt = ldw(a.count + j) + 1;
    // the committed node's old leaf per class: loaded (36 scattered lines) for one cluster; in a
    // sweep, where hundreds of scenarios share the caches, re-evaluated from the old row instead
    int32_t vold = -1;
    if (!a.nsc && cl) vold = ldw(a.leaves + cc * st0 + j);
    uint64_t gold[GL > 0 ? GL : 1];  // old global-level entries on the path
#pragma unroll
    for (int h = 1; h <= GL; ++h) gold[h - 1] = ldw(a.levels + s_off[h] + cc * s_st[h] + (e1 >> (6 * (h - 1))));
    kf64::FRow nr;
    nr.ac = (double)a.ac[j];
    nr.am = (double)a.am[j];
    nr.yc = a.ty[j];
    nr.ym = a.ty[n + j];
    nr.rc = (double)nrc; nr.rm = (double)nrm; nr.zc = (double)nzc; nr.zm = (double)nzm;
    nr.allowed = a.allowed[j];
    nr.count = ncnt;
    nr.fl = a.fl[j];
    uint32_t rmask;
    if (a.nsc) {
      kf64::FRow orow = nr;
      orow.rc = (double)(nrc - pc); orow.rm = (double)(nrm - pm); orow.zc = (double)(nzc - pzc);
      orow.zm = (double)(nzm - pzm); orow.count = ncnt - 1;
      const int32_t vo = kf64::feval(a.cfg, class_pod(s_cls[cc]), orow, rmask);
      vold = cl ? vo : -1;
    }
    const int32_t vnew = kf64::feval(a.cfg, class_pod(s_cls[cc]), nr, rmask);
    // stores only after every row load is consumed: stores and loads retire in issue order
    // (vmcnt), so a store issued ahead of the evaluation would make it wait for the store
    asm volatile("" ::"v"(vnew) : "memory");
    if (lane == 0) {
      a.out_node[p] = j;
      a.rc[j] = nrc; a.rm[j] = nrm; a.zc[j] = nzc; a.zm[j] = nzm; a.count[j] = ncnt;
    }
    const bool chg = cl && vnew != vold;
    TSTAMP(2);
    int resc_h = 0;       // level whose entry must be re-combined (0: none)
    uint64_t resc_old = 0;
    if (chg) {
      a.leaves[cc * st0 + j] = vnew;
      fitv += (vnew >= 0 ? 1 : 0) - (vold >= 0 ? 1 : 0);  // lane == class cc
    }
    {
      bool act = chg;
      uint64_t co = leaf_entry(vold), cn = leaf_entry(vnew);
#pragma unroll
      for (int h = 1; h <= ML; ++h) {
        if (h <= H && __ballot(act)) {
          const int eh = e1 >> (6 * (h - 1));
          if (act) {
            const uint64_t P = h <= GL ? gold[h <= GL ? h - 1 : 0] : kt_lds[s_off[h] + cc * s_st[h] + eh];
            uint64_t NP;
            if (!parent_rule(P, co, cn, NP)) {
              resc_h = h;
              resc_old = P;
              act = false;
            } else if (NP == P) {
              act = false;
            } else {
              if (h <= GL) a.levels[s_off[h] + cc * s_st[h] + eh] = NP;
              else kt_lds[s_off[h] + cc * s_st[h] + eh] = NP;
              if (h == H) rootv = NP;
              co = P;
              cn = NP;
            }
          }
        }
      }
    }
    // the rare paths whose unique maximum dropped: re-combine, then continue up (wave-wide)
    const uint64_t rmk = __ballot(resc_h != 0);
    if (rmk) stores_done();  // the leaves / entries just written are read back
    for (uint64_t rm = rmk; rm; rm &= rm - 1) {
      const int c = __builtin_ctzll(rm);
      int h = __builtin_amdgcn_readlane(resc_h, c);
      uint64_t oldv = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(resc_old >> 32), c) << 32) |
                      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)resc_old, c);
      uint64_t newv = rescan<M, GL>(a, s_st, s_off, c, h, e1 >> (6 * (h - 1)), lane);
      while (newv != oldv) {
        const int eh = e1 >> (6 * (h - 1));
        const int idx = s_off[h] + c * s_st[h] + eh;
        if (lane == 0) {
          if (h <= GL) a.levels[idx] = newv;
          else kt_lds[idx] = newv;
        }
        if (h == H) {
          if (lane == c) rootv = newv;
          break;
        }
        ++h;
        const int pidx = s_off[h] + c * s_st[h] + (e1 >> (6 * (h - 1)));
        const uint64_t P = h <= GL ? ldw(a.levels + pidx) : kt_lds[pidx];
        uint64_t NP;
        if (!parent_rule(P, oldv, newv, NP)) {
          stores_done();  // the children just written are read back by the re-combination
          NP = rescan<M, GL>(a, s_st, s_off, c, h, e1 >> (6 * (h - 1)), lane);
        }
        oldv = P;
        newv = NP;
      }
    }
#if KSIM_TREE_VAR == 2
    stores_done();
#endif
    TSTAMP(3);
#ifdef KSIM_STAMPS
    ts_acc[6] += __popcll(__ballot(chg));
    ts_acc[7] += __popcll(__ballot(resc_h != 0));
#endif
    hist_pod = -1;
    // quantities must stay exact in float64 (ksim_f64.h): stop after this pod otherwise
    stop = nrc >= LIM48 || nrm >= LIM48 || nzc >= LIM48 || nzm >= LIM48;
    ++p;
    if (lane == 0) __hip_atomic_store(&s_done, p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  if (lane == 0) __hip_atomic_store(&s_done, INT64_MAX, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  stores_done();
  for (int t = lane; t < lds_entries; t += 64) a.levels[gbase + t] = kt_lds[t];
  if (lane < K) a.fitc[lane] = fitv;
  if (lane == 0) {
    __hip_atomic_store(a.counter, counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.cursor, p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (stop) atomicOr(a.err, 8);
#ifdef KSIM_STAMPS
    for (int k = 0; k < 8; ++k) atomicAdd((unsigned long long*)&a.dbg[k], (unsigned long long)ts_acc[k]);
    atomicAdd((unsigned long long*)&a.dbg[8], (unsigned long long)(p - a.first));
#endif
  }
}

TreeArgs make_args(const KsimCtx* c, const KsimTreeGeo* g, const KsimTreeClass* cls, const int32_t* tcls,
                   int32_t* leaves, uint64_t* levels, int32_t* fitc, double* ty, const KsimTreeSweep* sw) {
  TreeArgs a{};
  a.g = *g;
  a.ac = c->alloc_cpu; a.am = c->alloc_mem;
  a.rc = c->req_cpu; a.rm = c->req_mem; a.zc = c->nz_cpu; a.zm = c->nz_mem;
  a.allowed = c->allowed_pods; a.count = c->pod_count; a.fl = c->flags;
  a.pods = c->pods; a.tcls = tcls; a.cls = cls;
  a.leaves = leaves; a.levels = levels; a.fitc = fitc; a.ty = ty;
  a.first = c->first; a.end = c->end;
  a.counter = c->counter; a.cursor = c->cursor; a.out_node = c->out_node; a.out_reasons = c->out_reasons;
  a.err = c->err;
  a.dbg = c->dbg;
  a.cfg = kf64::make_evcfg(c->preds, c->no_prio != 0, (int32_t)c->w[KSIM_W_LEAST_REQUESTED],
                           (int32_t)c->w[KSIM_W_MOST_REQUESTED], (int32_t)c->w[KSIM_W_BALANCED]);
  a.collect = c->collect;
  if (sw) {  // scenario sweep: per-scenario dynamic columns, counters, weights and outputs
    a.nsc = sw->nsc;
    a.rc = sw->rc; a.rm = sw->rm; a.zc = sw->zc; a.zm = sw->zm; a.count = sw->count;
    a.counter = sw->counter;
    a.out_node = sw->out_node;
    a.sw_cfg = (const kf64::EvCfg*)sw->cfg;
    a.sw_count = sw->count_pods;
    a.collect = 0;
  }
  return a;
}

}  // namespace

// scenario copies of the handle's dynamic columns and counter
__global__ __launch_bounds__(256) void ksim_tree_sweep_init_kernel(const int64_t* rc, const int64_t* rm, const int64_t* zc,
                                                                    const int64_t* zm, const int32_t* cnt, const uint64_t* ctr,
                                                                    int64_t n, KsimTreeSweep sw) {
  const int64_t tot = n * sw.nsc;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t % n;
    sw.rc[t] = rc[i]; sw.rm[t] = rm[i]; sw.zc[t] = zc[i]; sw.zm[t] = zm[i]; sw.count[t] = cnt[i];
    if (i == 0) sw.counter[t / n] = *ctr;
  }
}

extern "C" hipError_t ksim_tree_sweep_init(const KsimCtx* c, const KsimTreeSweep* sw, hipStream_t s) {
  const int64_t tot = c->n * sw->nsc;
  hipLaunchKernelGGL(ksim_tree_sweep_init_kernel, dim3((unsigned)std::min<int64_t>((tot + 255) / 256, 16384)), dim3(256), 0, s,
                     (const int64_t*)c->req_cpu, (const int64_t*)c->req_mem, (const int64_t*)c->nz_cpu,
                     (const int64_t*)c->nz_mem, (const int32_t*)c->pod_count, (const uint64_t*)c->counter, c->n, *sw);
  return hipGetLastError();
}

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
    if (H - hL > LS) continue;
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
                                      double* ty, const KsimTreeSweep* sw, hipStream_t s) {
  const TreeArgs a = make_args(c, g, cls, tcls, leaves, levels, fitc, ty, sw);
  const int nsc = a.nsc;
  const int64_t ns = std::max(1, nsc);
  const int64_t tl = (int64_t)g->K * g->st[0] * ns;
  hipLaunchKernelGGL(ksim_tree_leaf_kernel, dim3((unsigned)std::min<int64_t>((tl + 255) / 256, 8192)), dim3(256), 0, s, a);
  for (int h = 1; h <= g->H; ++h) {
    const int64_t waves = (int64_t)g->K * g->st[h] * ns;
    hipLaunchKernelGGL(ksim_tree_level_kernel, dim3((unsigned)std::min<int64_t>((waves + 3) / 4, 8192)), dim3(256), 0, s, a, h);
  }
  hipLaunchKernelGGL(ksim_tree_fit_kernel, dim3((unsigned)(g->K * ns)), dim3(256), 0, s, a);
  return hipGetLastError();
}

extern "C" hipError_t ksim_tree_launch(const KsimCtx* c, const KsimTreeGeo* g, const KsimTreeClass* cls,
                                       const int32_t* tcls, int32_t* leaves, uint64_t* levels, int32_t* fitc,
                                       double* ty, const KsimTreeSweep* sw, hipStream_t s) {
  const TreeArgs a = make_args(c, g, cls, tcls, leaves, levels, fitc, ty, sw);
  const unsigned grid = (unsigned)std::max(1, a.nsc);
  const size_t lds = (size_t)g->lds_entries * sizeof(uint64_t);
#define KT_CASE(MM, GG) \
  if (g->m == MM && g->hL == GG + 1) { hipLaunchKernelGGL((ksim_tree_kernel<MM, GG>), dim3(grid), dim3(128), lds, s, a); return hipGetLastError(); }
  KT_CASE(1, 0) KT_CASE(1, 1) KT_CASE(1, 2) KT_CASE(2, 0) KT_CASE(2, 1) KT_CASE(4, 0)
#undef KT_CASE
  return hipErrorInvalidValue;
}
