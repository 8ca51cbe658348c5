// ksim_sweep.hip — scenario sweep (BASELINE.json configs[4], SURVEY.md §8e "C5"): S independent
// copies of one cluster snapshot, each scheduling the same resource-only pod queue under its own
// map-priority weights — the capacity-planning what-if the reference answers by running the
// simulator once per policy (pkg/scheduler/simulator.go:286 New + :187 Run per
// --algorithmprovider / policy file).
//
// One 1024-thread workgroup per scenario; no cross-workgroup communication.  Per pod:
//   1. every thread evaluates rows j = tid, tid+1024, ... (coalesced), streaming the scenario's
//      dynamic columns (requested / non-zero requested cpu+mem as float64, pod count) from HBM
//      and the shared static columns (alloc, RN(1/alloc), allowed pods, flags) from L2; the
//      packed evaluation goes to LDS (uint16, 0xFFFF = does not fit);
//   2. block reduction → fit count F, max score M, count at max C (findNodesThatFit +
//      PrioritizeNodes, core/generic_scheduler.go:112-167);
//   3. selectHost (:183-198): ix = lastNodeIndex % C (no increment for a single fit node,
//      :153-156), the ix-th max-score row counted from the top of the name order, found by a
//      block prefix over contiguous LDS segments;
//   4. the owning thread commits (NodeInfo.AddPod, schedulercache/node_info.go:318-341) into the
//      scenario's columns; the barrier's workgroup fence makes it visible to the next pod.
// The node table streams from HBM every pod: the HBM-bandwidth-bound form of the scan.
#include "ksim_sweep.h"
#include "ksim_wave.h"

using namespace kf64;

namespace {
constexpr int SB = 1024;      // threads per scenario workgroup
constexpr int SW = SB / 64;   // waves
constexpr uint16_t NOFIT = 0xFFFF;
}  // namespace


__global__ __launch_bounds__(SB) void ksim_sweep_kernel(SwArgs a) {
  extern __shared__ uint16_t sc[];  // [n] evaluations of the current pod
  __shared__ int32_t s_red[SW][3];
  __shared__ int32_t s_wtot[SW];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int s = blockIdx.x;
  const int64_t n = a.n;
  const int64_t off = (int64_t)s * n;
  const int sw = a.scen0 + s;
  const EvCfg EC = make_evcfg(a.preds, a.no_prio != 0, a.w[3 * sw], a.w[3 * sw + 1], a.w[3 * sw + 2]);
  double* const rc = a.rc + off;
  double* const rm = a.rm + off;
  double* const zc = a.zc + off;
  double* const zm = a.zm + off;
  int32_t* const cnt = a.count + off;
  const int64_t K = (n + SB - 1) / SB;  // contiguous segment per thread in the select phase
  const int64_t seg0 = (int64_t)tid * K, seg1 = (seg0 + K < n) ? seg0 + K : n;
  uint64_t counter = a.counter0;  // genericScheduler.lastNodeIndex of this scenario

  for (int32_t p = 0; p < a.n_pods; ++p) {
    const FPod P = a.pods[p];
    // ---- 1. evaluate every row ----
    int32_t f = 0, mx = -1, cm = 0;
#pragma unroll 4
    for (int64_t j = tid; j < n; j += SB) {
      FRow r;
      r.ac = a.dac[j]; r.am = a.dam[j]; r.yc = a.yc[j]; r.ym = a.ym[j];
      r.rc = rc[j]; r.rm = rm[j]; r.zc = zc[j]; r.zm = zm[j];
      r.allowed = a.allowed[j]; r.count = cnt[j]; r.fl = a.flags[j];
      uint32_t rmask;
      const int32_t e = feval(EC, P, r, rmask);
      sc[j] = e < 0 ? NOFIT : (uint16_t)e;
      f += e >= 0 ? 1 : 0;
      cm = e > mx ? 1 : cm + ((e == mx && e >= 0) ? 1 : 0);
      mx = e > mx ? e : mx;
    }
    // ---- 2. block reduction: F, M, C ----
    {
      const int32_t Fw = ksimw::sum_i32(f);
      const int32_t Mw = ksimw::max_i32(mx);
      const int32_t Cw = ksimw::sum_i32((mx == Mw && mx >= 0) ? cm : 0);
      if (lane == 0) { s_red[wv][0] = Fw; s_red[wv][1] = Mw; s_red[wv][2] = Cw; }
    }
    __syncthreads();
    const bool in = lane < SW;
    const int32_t F = ksimw::sum_i32(in ? s_red[in ? lane : 0][0] : 0);
    const int32_t mw = in ? s_red[lane][1] : -1;
    const int32_t M = ksimw::max_i32(mw);
    const int32_t C = ksimw::sum_i32((in && mw == M && M >= 0) ? s_red[lane][2] : 0);
    if (F == 0) {  // FitError: no node fits
      if (tid == 0) a.out_node[(int64_t)s * a.n_pods + p] = -1;
      __syncthreads();  // s_red is rewritten by the next pod
      continue;
    }
    const uint32_t ix = (F > 1) ? (uint32_t)((counter >> 32) ? counter % (uint64_t)C : (uint32_t)counter % (uint32_t)C) : 0u;
    counter += (F > 1) ? 1 : 0;  // generic_scheduler.go:192-195 (selectHost only when F > 1)
    // ---- 3. the ix-th row at M from the top ----
    int32_t c_t = 0;
    for (int64_t j = seg0; j < seg1; ++j) c_t += (sc[j] == (uint16_t)M) ? 1 : 0;
    const int32_t pre = ksimw::prefix_incl_i32(c_t);  // within the wave
    if (lane == 63) s_wtot[wv] = pre;
    __syncthreads();
    int32_t below = 0;  // matches in lower waves
    for (int w = 0; w < SW; ++w) below += (w < wv) ? s_wtot[w] : 0;
    const uint32_t above = (uint32_t)(C - (below + pre));  // matches in higher threads
    if (c_t > 0 && ix >= above && ix < above + (uint32_t)c_t) {
      int32_t r = (int32_t)(ix - above);
      int64_t jsel = -1;
      for (int64_t j = seg1 - 1; j >= seg0; --j) {
        if (sc[j] == (uint16_t)M) {
          if (r == 0) { jsel = j; break; }
          --r;
        }
      }
      // ---- 4. commit ----
      if (jsel >= 0) {
        rc[jsel] += P.ad_c; rm[jsel] += P.ad_m; zc[jsel] += P.nz_c; zm[jsel] += P.nz_m; cnt[jsel] += 1;
      }
      a.out_node[(int64_t)s * a.n_pods + p] = (int32_t)jsel;
    }
    __syncthreads();  // the commit (workgroup release/acquire) before the next pod's loads
  }
  if (tid == 0) a.out_counter[s] = counter;
}

// static float64 columns, once per handle
__global__ void ksim_sweep_static_kernel(const int64_t* ac, const int64_t* am, int64_t n, double* dac, double* dam,
                                         double* yc, double* ym) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double c = (double)ac[i], m = (double)am[i];
  dac[i] = c; dam[i] = m;
  yc[i] = c != 0.0 ? 1.0 / c : 0.0;
  ym[i] = m != 0.0 ? 1.0 / m : 0.0;
}

// every scenario's dynamic columns from the handle's current node state
__global__ void ksim_sweep_init_kernel(const int64_t* rc0, const int64_t* rm0, const int64_t* zc0, const int64_t* zm0,
                                       const int32_t* c0, int64_t n, int64_t total, double* rc, double* rm, double* zc,
                                       double* zm, int32_t* c) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= total) return;
  const int64_t i = k % n;
  rc[k] = (double)rc0[i]; rm[k] = (double)rm0[i]; zc[k] = (double)zc0[i]; zm[k] = (double)zm0[i]; c[k] = c0[i];
}

__global__ void ksim_sweep_pods_kernel(const ksim_pod* pods, int64_t count, FPod* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) out[i] = load_fpod(pods[i]);
}

extern "C" size_t ksim_sweep_fpod_bytes(void) { return sizeof(FPod); }

extern "C" hipError_t ksim_sweep_prepare(const int64_t* ac, const int64_t* am, int64_t n, double* dac, double* dam,
                                         double* yc, double* ym, hipStream_t st) {
  hipLaunchKernelGGL(ksim_sweep_static_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ac, am, n, dac, dam,
                     yc, ym);
  return hipGetLastError();
}

extern "C" hipError_t ksim_sweep_launch(const int64_t* rc0, const int64_t* rm0, const int64_t* zc0, const int64_t* zm0,
                                        const int32_t* c0, const ksim_pod* pods, void* fpods, const SwArgs* args,
                                        int32_t n_scen, hipEvent_t ev0, hipEvent_t ev1, hipStream_t st) {
  const int64_t n = args->n, total = n * (int64_t)n_scen;
  hipLaunchKernelGGL(ksim_sweep_init_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, rc0, rm0, zc0, zm0,
                     c0, n, total, args->rc, args->rm, args->zc, args->zm, args->count);
  hipLaunchKernelGGL(ksim_sweep_pods_kernel, dim3((unsigned)((args->n_pods + 255) / 256)), dim3(256), 0, st, pods,
                     (int64_t)args->n_pods, (FPod*)fpods);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (ev0) (void)hipEventRecord(ev0, st);
  hipLaunchKernelGGL(ksim_sweep_kernel, dim3((unsigned)n_scen), dim3(SB), (size_t)n * sizeof(uint16_t), st, *args);
  e = hipGetLastError();
  if (ev1) (void)hipEventRecord(ev1, st);
  return e;
}
