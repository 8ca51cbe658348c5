// ksim_fast.h — per-node evaluation for "resource-only" pods (no host ports, no scalar or
// gpu/ephemeral request, no spec.nodeName, selector and tolerations that every label/taint
// set satisfies, one reduce class) — the C1/C3/C4/C5 pod shape.  Only the predicates that can
// fail for such a pod are evaluated, in predicatesOrdering order (predicates.go:129-138):
// CheckNodeCondition, CheckNodeUnschedulable, GeneralPredicates/PodFitsResources,
// CheckNodeMemoryPressure, CheckNodeDiskPressure.  (HostName, PodFitsHostPorts,
// MatchNodeSelector and PodToleratesNodeTaints pass by construction.)
//
// Scores in straight-line float64, still bit-exact, for requests and capacities below 2^49
// (larger operands take the int64 path of ksim_common.h):
//  * LeastRequested / MostRequested (least_requested.go:44-53, most_requested.go:45-55) are
//    floor(x / cap) with x = 10*(cap-req) or 10*req, integers below 2^53 and so exact in
//    float64.  The correctly rounded quotient never crosses an integer: if x/cap lies in
//    (k, k+1) then k+1 - x/cap >= 1/cap > 2^-49 >= ulp(k+1)/2 for k+1 <= 10, so truncating it
//    gives the int64 quotient.
//  * BalancedResourceAllocation (balanced_resource_allocation.go:39-61) is the reference's own
//    float64 expression (correctly rounded divides, no FMA contraction: -ffp-contract=off).
#pragma once
#include "ksim_common.h"

struct KsimFastPod {
  int64_t rq_c, rq_m;   // predicate request (GetResourceRequest)
  int64_t nz_c, nz_m;   // non-zero request (priorities)
  uint32_t flags;       // KSIM_POD_*
};

// One node row as the fast path needs it (dac/dam = alloc as float64, exact below 2^53).
struct KsimFastRow {
  int64_t ac, am, rc, rm, zc, zm;
  double dac, dam;
  int32_t allowed, count;
  uint32_t fl;
};

// Generic (divide-based) weighted score: operands at or beyond 2^49, kept out of line.
__device__ __noinline__ int64_t ksim_slow_score(int64_t tc, int64_t ac, int64_t tm, int64_t am, int64_t wl, int64_t wm,
                                                int64_t wb) {
  uint64_t s = 0;
  if (wl) s += (uint64_t)wl * (uint64_t)((ksim_least(tc, ac) + ksim_least(tm, am)) / 2);
  if (wm) s += (uint64_t)wm * (uint64_t)((ksim_most(tc, ac) + ksim_most(tm, am)) / 2);
  if (wb) s += (uint64_t)wb * (uint64_t)ksim_balanced(tc, ac, tm, am);
  return (int64_t)s;
}

// Weighted map score (LR/MR/BRA) of one node: tc/tm = pod non-zero request + node non-zero
// requested (resource_allocation.go:58-59).
__device__ __forceinline__ int64_t ksim_fast_score(int64_t tc, int64_t ac, double dac, int64_t tm, int64_t am, double dam,
                                                   int64_t wl, int64_t wm, int64_t wb) {
  if (((uint64_t)(tc | ac | tm | am)) >> 49) return ksim_slow_score(tc, ac, tm, am, wl, wm, wb);
  const double xc = (double)tc, xm = (double)tm;
  const bool okc = ac != 0 && tc <= ac, okm = am != 0 && tm <= am;
  const double bc = ac ? dac : 1.0, bm = am ? dam : 1.0;
  int64_t s = 0;
  if (wl) {
    const int32_t lc = okc ? (int32_t)((bc - xc) * 10.0 / bc) : 0;
    const int32_t lm = okm ? (int32_t)((bm - xm) * 10.0 / bm) : 0;
    s += wl * ((lc + lm) / 2);
  }
  if (wm) {
    const int32_t mc = okc ? (int32_t)(xc * 10.0 / bc) : 0;
    const int32_t mm = okm ? (int32_t)(xm * 10.0 / bm) : 0;
    s += wm * ((mc + mm) / 2);
  }
  if (wb) {
    const double fc = ac ? xc / bc : 1.0;
    const double fm = am ? xm / bm : 1.0;
    const int32_t b = (fc >= 1.0 || fm >= 1.0) ? 0 : (int32_t)((1.0 - fabs(fc - fm)) * 10.0);
    s += wb * b;
  }
  return s;
}

// Reason mask of the first failing predicate (0 = fits) for a resource-only pod.
__device__ __forceinline__ uint32_t ksim_fast_predicates(uint32_t preds, const KsimFastPod& P, int64_t ac,
                                                         int64_t am, int64_t rc, int64_t rm, int32_t allowed,
                                                         int32_t count, uint32_t fl) {
  // evaluated branch-free, then the first failing predicate in order wins
  const uint32_t cond = (preds & KSIM_P_CHECK_NODE_CONDITION) ? (fl & KSIM_COND_REASON_MASK) : 0u;
  const uint32_t unsch =
      ((preds & KSIM_P_CHECK_NODE_UNSCHEDULABLE) && (fl & KSIM_N_UNSCHEDULABLE)) ? (1u << KSIM_R_UNSCHEDULABLE) : 0u;
  uint32_t res = 0;
  if (preds & (KSIM_P_GENERAL | KSIM_P_RESOURCES)) {
    res = (count + 1 > allowed) ? (1u << KSIM_R_INSUFFICIENT_PODS) : 0u;
    if (P.flags & KSIM_POD_ANY_REQUEST) {
      res |= (ac < P.rq_c + rc) ? (1u << KSIM_R_INSUFFICIENT_CPU) : 0u;
      res |= (am < P.rq_m + rm) ? (1u << KSIM_R_INSUFFICIENT_MEMORY) : 0u;
      res |= (fl & KSIM_N_GPU_OVER) ? (1u << KSIM_R_INSUFFICIENT_GPU) : 0u;
      res |= (fl & KSIM_N_EPH_OVER) ? (1u << KSIM_R_INSUFFICIENT_EPHEMERAL) : 0u;
    }
  }
  const uint32_t lp = ((preds & KSIM_P_LABEL_PRESENCE) && (fl & KSIM_N_LABEL_PRESENCE)) ? (1u << KSIM_R_LABEL_PRESENCE) : 0u;
  const uint32_t memp = ((preds & KSIM_P_MEM_PRESSURE) && (P.flags & KSIM_POD_BEST_EFFORT) && (fl & KSIM_N_MEM_PRESSURE))
                            ? (1u << KSIM_R_MEM_PRESSURE)
                            : 0u;
  const uint32_t diskp = ((preds & KSIM_P_DISK_PRESSURE) && (fl & KSIM_N_DISK_PRESSURE)) ? (1u << KSIM_R_DISK_PRESSURE) : 0u;
  return cond ? cond : unsch ? unsch : res ? res : lp ? lp : memp ? memp : diskp;
}

// Packed evaluation of a row for a resource-only pod (-1 = does not fit, else the score) and
// its reason mask.
__device__ __forceinline__ int32_t ksim_fast_eval(uint32_t preds, const KsimFastPod& F, const KsimFastRow& r,
                                                  bool no_prio, int64_t wl, int64_t wm, int64_t wb, uint32_t& rm) {
  const uint32_t m = ksim_fast_predicates(preds, F, r.ac, r.am, r.rc, r.rm, r.allowed, r.count, r.fl);
  rm = m;
  const int32_t sc =
      no_prio ? 0 : (int32_t)ksim_fast_score(F.nz_c + r.zc, r.ac, r.dac, F.nz_m + r.zm, r.am, r.dam, wl, wm, wb);
  return m ? -1 : sc;
}

// Does pod P qualify for the fast path under this configuration?
__device__ __forceinline__ bool ksim_is_fast_pod(const ksim_pod& P, int K) {
  return K == 1 && P.host == -1 && P.port_cnt == 0 && P.scalar_cnt == 0 && P.req_gpu == 0 && P.req_eph == 0 &&
         !(P.flags & (KSIM_POD_NEED_SELECTOR | KSIM_POD_NEED_TAINTS));
}
