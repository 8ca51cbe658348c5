// ksim_cache.hip — device side of the scheduler-cache event mirror (ksim_cache.cpp).
//
// The Go scheduler keeps its node cache in sync with the cluster through informer events
// (pkg/scheduler/factory/factory.go:596 addPodToCache, :740 addNodeToCache, feeding
// schedulercache/cache.go AddPod / RemovePod / AddNode / UpdateNode / RemoveNode).  Here the
// cache is the HBM-resident name-ranked node table, so every event is a small kernel:
//   * node add / remove  — relayout: every column is copied once into a table one row longer
//     or shorter (rows keep their name-rank order), one launch for all columns;
//   * node add / update  — set_row: NodeInfo.SetNode's static columns (and, on add, the
//     dynamic ones) from a packed row, over-commit bits re-derived;
//   * pod add / remove   — NodeInfo.AddPod / RemovePod on one row (ksim_commit / ksim_uncommit);
//   * queued pods' spec.nodeName indices follow the shifted name ranks (remap_hosts).
// All of it is integer / byte movement: HBM-bound copies, no arithmetic worth an MFMA.
#include "ksim_common.h"
#include "ksim_cache.h"

__global__ __launch_bounds__(256) void ksim_relayout_kernel(KsimRelayout r) {
  const KsimRelayCol col = r.col[blockIdx.y];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < r.n_new; j += stride) {
    int64_t src = j;
    if (r.op == KSIM_RELAY_INSERT) src = j < r.idx ? j : (j == r.idx ? -1 : j - 1);
    else if (r.op == KSIM_RELAY_REMOVE) src = j < r.idx ? j : j + 1;
    for (int32_t k = 0; k < col.dst_slots; ++k) {
      const bool have = src >= 0 && k < col.src_slots;
      if (col.esz == 8) {
        const uint64_t v = have ? static_cast<const uint64_t*>(col.src)[k * r.n_old + src] : 0ull;
        static_cast<uint64_t*>(col.dst)[k * r.n_new + j] = v;
      } else {
        const uint32_t v = have ? static_cast<const uint32_t*>(col.src)[k * r.n_old + src] : 0u;
        static_cast<uint32_t*>(col.dst)[k * r.n_new + j] = v;
      }
    }
  }
}

// NodeInfo.SetNode (node_info.go:429-448) on row i: allocatable, allowed pods, condition bits,
// label / taint set; with `full` also the dynamic columns (a node added with pods already on
// it).  The over-commit bits are re-derived from allocatable vs requested.  Single thread.
__global__ void ksim_set_row_kernel(KsimCtx c, int64_t i, const uint64_t* __restrict__ pk, int32_t full) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int64_t n = c.n;
  const_cast<int64_t*>(c.alloc_cpu)[i] = (int64_t)pk[KSIM_PK_ALLOC + 0];
  const_cast<int64_t*>(c.alloc_mem)[i] = (int64_t)pk[KSIM_PK_ALLOC + 1];
  const int64_t ag = (int64_t)pk[KSIM_PK_ALLOC + 2], ae = (int64_t)pk[KSIM_PK_ALLOC + 3];
  const_cast<int64_t*>(c.alloc_gpu)[i] = ag;
  const_cast<int64_t*>(c.alloc_eph)[i] = ae;
  const_cast<int32_t*>(c.allowed_pods)[i] = (int32_t)pk[KSIM_PK_ALLOWED];
  const_cast<int32_t*>(c.label_set)[i] = (int32_t)pk[KSIM_PK_LABEL];
  const_cast<int32_t*>(c.taint_set)[i] = (int32_t)pk[KSIM_PK_TAINT];
  for (int32_t k = 0; k < c.n_scalar; ++k) const_cast<int64_t*>(c.alloc_scalar)[k * n + i] = (int64_t)pk[KSIM_PK_SCALAR + k];
  if (full) {
    c.req_cpu[i] = (int64_t)pk[KSIM_PK_REQ + 0];
    c.req_mem[i] = (int64_t)pk[KSIM_PK_REQ + 1];
    c.req_gpu[i] = (int64_t)pk[KSIM_PK_REQ + 2];
    c.req_eph[i] = (int64_t)pk[KSIM_PK_REQ + 3];
    c.nz_cpu[i] = (int64_t)pk[KSIM_PK_NZ + 0];
    c.nz_mem[i] = (int64_t)pk[KSIM_PK_NZ + 1];
    c.pod_count[i] = (int32_t)pk[KSIM_PK_COUNT];
    for (int32_t k = 0; k < c.n_scalar; ++k) c.req_scalar[k * n + i] = (int64_t)pk[KSIM_PK_SCALAR + c.n_scalar + k];
    const int32_t pc = (int32_t)pk[KSIM_PK_PORTCNT];
    for (int32_t k = 0; k < c.port_slots; ++k) c.ports[k * n + i] = k < pc ? pk[KSIM_PK_SCALAR + 2 * c.n_scalar + k] : 0ull;
    if (c.port_slots) c.port_count[i] = pc;
  }
  uint32_t f = (uint32_t)pk[KSIM_PK_FLAGS] & 0xFFu;
  if (ag < c.req_gpu[i]) f |= KSIM_N_GPU_OVER;
  if (ae < c.req_eph[i]) f |= KSIM_N_EPH_OVER;
  c.flags[i] = f;
}

// NodeInfo.RemovePod of queue pod `pod` from row `node` (ksim_pod_remove).
__global__ void ksim_release_kernel(KsimCtx c, int64_t pod, int64_t node) {
  if (blockIdx.x != 0 || threadIdx.x >= 64) return;
  ksim_pod P;  // (a branch, not a pointer select: the pod stays in registers)
  if (c.one) P = c.one_pod;
  else P = c.pods[pod];
  if (threadIdx.x == 0) {
    ksim_uncommit(c, P, node);
    if (ksim_is_vol_pod(c, P)) ksim_vol_commit_body(*c.vol, P, node, -1, c.err);
  }
  if (ksim_is_aff_pod(c, P)) ksim_aff_commit_body(*c.aff, P, node, -1, threadIdx.x, 64);
}

// Undo a tentative commit whose record left with the resident kernel (ksim_cache.cpp).
__global__ void ksim_undo_kernel(KsimCtx c, KsimTentRec t) {
  if (blockIdx.x != 0 || threadIdx.x >= 64) return;
  if (threadIdx.x == 0) {
    ksim_undo_commit(c, t);
    if (ksim_is_vol_pod(c, t.P)) ksim_vol_commit_body(*c.vol, t.P, t.node, -1, c.err);
  }
  if (ksim_is_aff_pod(c, t.P)) ksim_aff_commit_body(*c.aff, t.P, t.node, -1, threadIdx.x, 64);
}

// Queued pods' spec.nodeName name ranks after a node insert (op 1) or removal (op 2).
__global__ __launch_bounds__(256) void ksim_remap_hosts_kernel(ksim_pod* pods, int64_t n_pods, int64_t idx, int32_t op) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_pods; p += stride) {
    const int32_t h = pods[p].host;
    if (h < 0) continue;
    if (op == KSIM_RELAY_INSERT) {
      if (h >= idx) pods[p].host = h + 1;
    } else if (op == KSIM_RELAY_REMOVE) {
      if (h == idx) pods[p].host = -2;  // names a node that is no longer listed
      else if (h > idx) pods[p].host = h - 1;
    }
  }
}

__global__ __launch_bounds__(256) void ksim_port_max_kernel(const int32_t* __restrict__ pc, int64_t n, int32_t* out) {
  int32_t m = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) m = pc[i] > m ? pc[i] : m;
  for (int o = 32; o > 0; o >>= 1) {
    const int32_t t = __shfl_xor(m, o, 64);
    m = t > m ? t : m;
  }
  if ((threadIdx.x & 63) == 0 && m) atomicMax(out, m);
}

// Per queued pod, its reduce-class counts k1 (TaintToleration) / k2 (NodeAffinity) into
// reserved[0..1] (1 when the priority is not configured), read by the persistent kernel's
// descriptor ring instead of the class tables.
__global__ __launch_bounds__(256) void ksim_pod_k_kernel(ksim_pod* pods, int64_t n_pods, const int32_t* __restrict__ n_tt,
                                                         const int32_t* __restrict__ n_na, int32_t use_tt, int32_t use_na) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_pods; p += stride) {
    const int32_t cls = pods[p].cls;
    pods[p].reserved[0] = use_tt ? n_tt[cls] : 1;
    pods[p].reserved[1] = use_na ? n_na[cls] : 1;
  }
}

static int grid_for(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

extern "C" hipError_t ksim_launch_relayout(const KsimRelayout* r, hipStream_t s) {
  if (r->ncol <= 0) return hipSuccess;
  hipLaunchKernelGGL(ksim_relayout_kernel, dim3(grid_for(r->n_new), r->ncol), dim3(256), 0, s, *r);
  return hipGetLastError();
}

extern "C" hipError_t ksim_launch_set_row(const KsimCtx* c, int64_t node, const uint64_t* pack, int32_t full,
                                          hipStream_t s) {
  hipLaunchKernelGGL(ksim_set_row_kernel, dim3(1), dim3(64), 0, s, *c, node, pack, full);
  return hipGetLastError();
}

extern "C" hipError_t ksim_launch_undo(const KsimCtx* c, const KsimTentRec* t, hipStream_t s) {
  if (t->node < 0 || t->node >= c->n) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ksim_undo_kernel, dim3(1), dim3(64), 0, s, *c, *t);
  return hipGetLastError();
}

extern "C" hipError_t ksim_launch_release(const KsimCtx* c, int64_t pod, int64_t node, hipStream_t s) {
  hipLaunchKernelGGL(ksim_release_kernel, dim3(1), dim3(64), 0, s, *c, pod, node);
  return hipGetLastError();
}

extern "C" hipError_t ksim_launch_remap_hosts(ksim_pod* pods, int64_t n_pods, int64_t idx, int32_t op, hipStream_t s) {
  if (n_pods <= 0) return hipSuccess;
  hipLaunchKernelGGL(ksim_remap_hosts_kernel, dim3(grid_for(n_pods)), dim3(256), 0, s, pods, n_pods, idx, op);
  return hipGetLastError();
}

extern "C" hipError_t ksim_launch_port_max(const int32_t* port_count, int64_t n, int32_t* out, hipStream_t s) {
  hipError_t e = hipMemsetAsync(out, 0, 4, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(ksim_port_max_kernel, dim3(grid_for(n)), dim3(256), 0, s, port_count, n, out);
  return hipGetLastError();
}

extern "C" hipError_t ksim_launch_pod_k(ksim_pod* pods, int64_t n_pods, const KsimCtx* c, hipStream_t s) {
  if (n_pods <= 0) return hipSuccess;
  hipLaunchKernelGGL(ksim_pod_k_kernel, dim3(grid_for(n_pods)), dim3(256), 0, s, pods, n_pods, c->n_tt, c->n_na,
                     c->w[KSIM_W_TAINT_TOLERATION] != 0 ? 1 : 0, c->use_na);
  return hipGetLastError();
}
