// ksim_f64.h — float64 evaluation of resource-only pods (ksim_is_fast_pod) shared by the
// fast persistent kernel (ksim_pfast.hip) and the scenario-sweep kernel (ksim_sweep.hip).
//
// Every cpu / memory quantity is an integer below 2^48 and every sum below 2^49 (host and
// in-kernel checks), so sums, compares and the products below are exact in float64 and the
// Go int64 arithmetic is reproduced without 64-bit integer emulation.  Each row carries
// y = RN(1/alloc) (alloc is static):
//  * LeastRequested / MostRequested floor(10x / cap) (least_requested.go:44-53,
//    most_requested.go:45-55) = trunc(x*y) corrected by the exact remainder fma(-q, cap, x);
//  * BalancedResourceAllocation's float64(req)/float64(cap) (balanced_resource_allocation.go:
//    39-61) = Markstein's RN(a/b): q = a*y, r = fma(-q, b, a) (exact), RN(q + r*y) — the
//    correctly rounded quotient, bit-identical to the IEEE divide Go performs (y within half an
//    ulp of 1/b, q within one ulp of a/b, no over/underflow).
#pragma once
#include "ksim_common.h"

namespace kf64 {

struct FRow {
  double ac, am, rc, rm, zc, zm, yc, ym;  // y = RN(1/alloc) (0 when alloc == 0)
  int32_t allowed, count;
  uint32_t fl;
};

// the pod fields the fast path reads, as float64 (wave-uniform)
struct FPod {
  double rq_c, rq_m, nz_c, nz_m, ad_c, ad_m;
  uint32_t anyreq;  // ~0u when PodFitsResources does the resource checks (predicates.go:731-736)
  uint32_t be;      // ~0u for a BestEffort pod (CheckNodeMemoryPressure, predicates.go:1502)
};

// the configured predicate set and weights as masks / multipliers (no branches per row)
struct EvCfg {
  uint32_t condm;   // node-condition bits checked (CheckNodeCondition)
  uint32_t unschm;  // KSIM_N_UNSCHEDULABLE if CheckNodeUnschedulable is configured
  uint32_t resm;    // ~0u if PodFitsResources runs (GeneralPredicates / PodFitsResources)
  uint32_t mempm;   // KSIM_N_MEM_PRESSURE if CheckNodeMemoryPressure is configured
  uint32_t diskm;   // KSIM_N_DISK_PRESSURE if CheckNodeDiskPressure is configured
  uint32_t lpm;     // KSIM_N_LABEL_PRESENCE if CheckNodeLabelPresence is configured
  int32_t wl, wm, wb;  // 0 for every weight under an empty prioritizer list (EqualPriorityMap)
};

__host__ __device__ inline EvCfg make_evcfg(uint32_t preds, bool no_prio, int32_t wl, int32_t wm, int32_t wb) {
  EvCfg C;
  C.condm = (preds & KSIM_P_CHECK_NODE_CONDITION) ? KSIM_COND_REASON_MASK : 0u;
  C.unschm = (preds & KSIM_P_CHECK_NODE_UNSCHEDULABLE) ? KSIM_N_UNSCHEDULABLE : 0u;
  C.resm = (preds & (KSIM_P_GENERAL | KSIM_P_RESOURCES)) ? ~0u : 0u;
  C.mempm = (preds & KSIM_P_MEM_PRESSURE) ? KSIM_N_MEM_PRESSURE : 0u;
  C.diskm = (preds & KSIM_P_DISK_PRESSURE) ? KSIM_N_DISK_PRESSURE : 0u;
  C.lpm = (preds & KSIM_P_LABEL_PRESENCE) ? KSIM_N_LABEL_PRESENCE : 0u;
  C.wl = no_prio ? 0 : wl;
  C.wm = no_prio ? 0 : wm;
  C.wb = no_prio ? 0 : wb;
  return C;
}

__device__ __forceinline__ FPod load_fpod(const ksim_pod& P) {
  return FPod{(double)P.req_cpu, (double)P.req_mem, (double)P.nz_cpu, (double)P.nz_mem,
              (double)P.add_cpu, (double)P.add_mem, (P.flags & KSIM_POD_ANY_REQUEST) ? ~0u : 0u,
              (P.flags & KSIM_POD_BEST_EFFORT) ? ~0u : 0u};
}

// row + pod (NodeInfo.AddPod, node_info.go:318-341, the columns the fast path keeps)
__device__ __forceinline__ FRow plus(FRow r, const FPod& P) {
  r.rc += P.ad_c; r.rm += P.ad_m; r.zc += P.nz_c; r.zm += P.nz_m; r.count += 1;
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

// Packed evaluation (-1 = does not fit, else the weighted map score) and reason mask of
// one row, straight-line (a taken branch costs a single wave ~40 cycles): predicates in
// predicatesOrdering order as ksim_fast_predicates — the first failing one's reason — then
// LeastRequested / MostRequested / BalancedResourceAllocation on tc/tm = pod non-zero request
// + node non-zero requested (resource_allocation.go:58-59), all three computed and weighted
// (a weight of 0 drops a priority).
__device__ __forceinline__ int32_t feval(const EvCfg& C, const FPod& P, const FRow& r, uint32_t& rmask) {
  const uint32_t fl = r.fl;
  const uint32_t cond = fl & C.condm;  // bit positions coincide with KSIM_R_*
  const uint32_t unsch = (fl & C.unschm) ? (1u << KSIM_R_UNSCHEDULABLE) : 0u;
  uint32_t rq = (r.ac < P.rq_c + r.rc) ? (1u << KSIM_R_INSUFFICIENT_CPU) : 0u;
  rq |= (r.am < P.rq_m + r.rm) ? (1u << KSIM_R_INSUFFICIENT_MEMORY) : 0u;
  rq |= (fl & KSIM_N_GPU_OVER) ? (1u << KSIM_R_INSUFFICIENT_GPU) : 0u;
  rq |= (fl & KSIM_N_EPH_OVER) ? (1u << KSIM_R_INSUFFICIENT_EPHEMERAL) : 0u;
  const uint32_t res = (((r.count + 1 > r.allowed) ? (1u << KSIM_R_INSUFFICIENT_PODS) : 0u) | (rq & P.anyreq)) & C.resm;
  const uint32_t memp = (fl & C.mempm & P.be) ? (1u << KSIM_R_MEM_PRESSURE) : 0u;
  const uint32_t diskp = (fl & C.diskm) ? (1u << KSIM_R_DISK_PRESSURE) : 0u;
  const uint32_t lp = (fl & C.lpm) ? (1u << KSIM_R_LABEL_PRESENCE) : 0u;
  const uint32_t m = cond ? cond : unsch ? unsch : res ? res : lp ? lp : memp ? memp : diskp;
  rmask = m;
  const double tc = P.nz_c + r.zc, tm = P.nz_m + r.zm;
  const bool okc = r.ac != 0.0 && tc <= r.ac, okm = r.am != 0.0 && tm <= r.am;
  const int32_t lc = div_floor((r.ac - tc) * 10.0, r.ac, r.yc), lm = div_floor((r.am - tm) * 10.0, r.am, r.ym);
  const int32_t mc = div_floor(tc * 10.0, r.ac, r.yc), mm = div_floor(tm * 10.0, r.am, r.ym);
  const uint32_t lr = ((uint32_t)(okc ? lc : 0) + (uint32_t)(okm ? lm : 0)) >> 1;
  const uint32_t mr = ((uint32_t)(okc ? mc : 0) + (uint32_t)(okm ? mm : 0)) >> 1;
  const double qc = quot(tc, r.ac, r.yc), qm = quot(tm, r.am, r.ym);
  const double fc = r.ac != 0.0 ? qc : 1.0, fm = r.am != 0.0 ? qm : 1.0;
  const int32_t bt = (int32_t)((1.0 - fabs(fc - fm)) * 10.0);
  const int32_t br = (fc >= 1.0 || fm >= 1.0) ? 0 : bt;
  const int32_t sc = C.wl * (int32_t)lr + C.wm * (int32_t)mr + C.wb * br;
  return m ? -1 : sc;
}

}  // namespace kf64
