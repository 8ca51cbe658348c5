// ksim_fast.h — per-node evaluation for "resource-only" pods (no host ports, no scalar or
// gpu/ephemeral request, no spec.nodeName, selector and tolerations that every label/taint
// set satisfies, one reduce class) — the C1/C3/C4/C5 pod shape.  Only the predicates that can
// fail for such a pod are evaluated, in predicatesOrdering order (predicates.go:129-138):
// CheckNodeCondition, CheckNodeUnschedulable, GeneralPredicates/PodFitsResources,
// CheckNodeMemoryPressure, CheckNodeDiskPressure.  (HostName, PodFitsHostPorts,
// MatchNodeSelector and PodToleratesNodeTaints pass by construction.)
//
// Scores without a divide on the common path, still bit-exact:
//  * LeastRequested / MostRequested (least_requested.go:44-53, most_requested.go:45-55) are
//    floor(10*(cap-req)/cap) and floor(10*req/cap) in int64: an estimate from a per-node
//    reciprocal is off by at most one and is corrected with two int64 multiplies.
//  * BalancedResourceAllocation (balanced_resource_allocation.go:39-61) truncates
//    (1-|fc-fm|)*10 computed from correctly rounded fc = req/cap, fm.  The reciprocal estimate
//    is within ~1e-14 of the real value; whenever it is farther than 1e-9 from an integer (and
//    from the fc/fm >= 1 boundary) the truncation equals the reference's, otherwise the exact
//    IEEE divide sequence runs.
#pragma once
#include "ksim_common.h"

struct KsimFastPod {
  int64_t rq_c, rq_m;   // predicate request (GetResourceRequest)
  int64_t nz_c, nz_m;   // non-zero request (priorities)
  uint32_t flags;       // KSIM_POD_*
};

__device__ __forceinline__ int64_t ksim_fix_q(int32_t q, int64_t x, int64_t b) {
  // q in [0, 11] approximates floor(x / b), 0 <= x < 2^53, 0 < b < 2^49, |error| <= 1
  q = q < 0 ? 0 : q;
  const int64_t qb = (int64_t)q * b;
  if (qb > x) return q - 1;
  if (qb + b <= x) return q + 1;
  return q;
}

__device__ __noinline__ int64_t ksim_bra_exact(int64_t tc, int64_t ac, int64_t tm, int64_t am) {
  return ksim_balanced(tc, ac, tm, am);
}

// Generic (divide-based) weighted score: operands beyond 2^49, kept out of line.
__device__ __noinline__ int64_t ksim_slow_score(int64_t tc, int64_t ac, int64_t tm, int64_t am, int64_t wl, int64_t wm,
                                                int64_t wb) {
  uint64_t s = 0;
  if (wl) s += (uint64_t)wl * (uint64_t)((ksim_least(tc, ac) + ksim_least(tm, am)) / 2);
  if (wm) s += (uint64_t)wm * (uint64_t)((ksim_most(tc, ac) + ksim_most(tm, am)) / 2);
  if (wb) s += (uint64_t)wb * (uint64_t)ksim_balanced(tc, ac, tm, am);
  return (int64_t)s;
}

// Weighted map score (LR/MR/BRA) of one node; inv_* = 1.0 / alloc (0 when alloc == 0).
__device__ __forceinline__ int64_t ksim_fast_score(int64_t tc, int64_t ac, double ic, int64_t tm, int64_t am, double im,
                                                   int64_t wl, int64_t wm, int64_t wb) {
  if (((tc | ac | tm | am) >> 49) != 0 || tc < 0 || tm < 0) return ksim_slow_score(tc, ac, tm, am, wl, wm, wb);
  const double fc = ac ? (double)tc * ic : 1.0;  // estimates of req / cap
  const double fm = am ? (double)tm * im : 1.0;
  int64_t s = 0;
  if (wl | wm) {
    int64_t lc = 0, lm = 0, mc = 0, mm = 0;
    if (ac != 0 && tc <= ac) {
      lc = ksim_fix_q((int32_t)(10.0 - 10.0 * fc), (ac - tc) * 10, ac);
      mc = ksim_fix_q((int32_t)(10.0 * fc), tc * 10, ac);
    }
    if (am != 0 && tm <= am) {
      lm = ksim_fix_q((int32_t)(10.0 - 10.0 * fm), (am - tm) * 10, am);
      mm = ksim_fix_q((int32_t)(10.0 * fm), tm * 10, am);
    }
    s += wl * ((lc + lm) / 2) + wm * ((mc + mm) / 2);
  }
  if (wb) {
    int64_t b;
    const bool near_one = fabs(fc - 1.0) < 1e-12 || fabs(fm - 1.0) < 1e-12;
    if (near_one) {
      b = ksim_bra_exact(tc, ac, tm, am);
    } else if (fc >= 1.0 || fm >= 1.0) {
      b = 0;
    } else {
      const double v = (1.0 - fabs(fc - fm)) * 10.0;
      const double fl = floor(v);
      const double fr = v - fl;
      b = (fr < 1e-9 || fr > 1.0 - 1e-9) ? ksim_bra_exact(tc, ac, tm, am) : (int64_t)fl;
    }
    s += wb * b;
  }
  return s;
}

// Reason mask of the first failing predicate (0 = fits) for a resource-only pod.
__device__ __forceinline__ uint32_t ksim_fast_predicates(uint32_t preds, const KsimFastPod& P, int64_t ac,
                                                         int64_t am, int64_t rc, int64_t rm, int32_t allowed,
                                                         int32_t count, uint32_t fl) {
  if (preds & KSIM_P_CHECK_NODE_CONDITION) {
    const uint32_t m = fl & KSIM_COND_REASON_MASK;
    if (m) return m;
  }
  if ((preds & KSIM_P_CHECK_NODE_UNSCHEDULABLE) && (fl & KSIM_N_UNSCHEDULABLE)) return 1u << KSIM_R_UNSCHEDULABLE;
  if (preds & (KSIM_P_GENERAL | KSIM_P_RESOURCES)) {
    uint32_t m = (count + 1 > allowed) ? (1u << KSIM_R_INSUFFICIENT_PODS) : 0u;
    if (P.flags & KSIM_POD_ANY_REQUEST) {
      if (ac < P.rq_c + rc) m |= 1u << KSIM_R_INSUFFICIENT_CPU;
      if (am < P.rq_m + rm) m |= 1u << KSIM_R_INSUFFICIENT_MEMORY;
      if (fl & KSIM_N_GPU_OVER) m |= 1u << KSIM_R_INSUFFICIENT_GPU;
      if (fl & KSIM_N_EPH_OVER) m |= 1u << KSIM_R_INSUFFICIENT_EPHEMERAL;
    }
    if (m) return m;
  }
  if ((preds & KSIM_P_MEM_PRESSURE) && (P.flags & KSIM_POD_BEST_EFFORT) && (fl & KSIM_N_MEM_PRESSURE))
    return 1u << KSIM_R_MEM_PRESSURE;
  if ((preds & KSIM_P_DISK_PRESSURE) && (fl & KSIM_N_DISK_PRESSURE)) return 1u << KSIM_R_DISK_PRESSURE;
  return 0;
}

// Does pod P qualify for the fast path under this configuration?
__device__ __forceinline__ bool ksim_is_fast_pod(const ksim_pod& P, int K) {
  return K == 1 && P.host == -1 && P.port_cnt == 0 && P.scalar_cnt == 0 && P.req_gpu == 0 && P.req_eph == 0 &&
         !(P.flags & (KSIM_POD_NEED_SELECTOR | KSIM_POD_NEED_TAINTS));
}
