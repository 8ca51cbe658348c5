// ksim_persistent.hip — persistent-kernel mode (KSIM_MODE_PERSISTENT).
//
// One launch walks the whole pod queue.  Workgroup b owns the contiguous name-rank range
// [b*chunk, (b+1)*chunk) of the node table and keeps the hot 60-byte rows of those nodes in
// LDS for the whole launch (only the owner of a node ever reads or writes it, so node state
// needs no cross-workgroup coherence).  Per pod p:
//   a. every workgroup publishes its partial for p — fit count + per reduce class (max map
//      score, count at max) — as tagged 8-byte granules (one agent-scope store each: the data
//      is the flag; MI355X_MICROARCH.md "handoff-1to1" / "allgather");
//   b. it evaluates pod p+1 against its rows SPECULATIVELY (assuming p's winner is not in its
//      range — true for all but one workgroup) while the other partials of p arrive;
//   c. one wave per workgroup sweeps every workgroup's granules for p and computes the global
//      decision redundantly (findNodesThatFit → PrioritizeNodes → selectHost,
//      core/generic_scheduler.go:112-198, lastNodeIndex replicated in every workgroup) — no
//      second exchange, no grid barrier;
//   d. the owner of the selected range picks the exact node from the p scores it still holds
//      in registers, commits the pod into LDS (NodeInfo.AddPod) and re-evaluates only that
//      row for p+1, fixing its speculative partial.
// The critical path per pod is therefore publish → sweep → decide → one-row fix-up; the
// full-table evaluation of the next pod overlaps the exchange.
// Granules are double-buffered by pod parity with an 8-bit pod tag: a workgroup that publishes
// pod p has seen every workgroup's pod p-1 partial, so nobody still reads the p-2 slot it
// overwrites.  Every spin is bounded (2 s) and reports through the error word.
//
// Granule q of a workgroup: tag:8 | fit:12 (q = 0 only) | count:12 | score:32 (class q max,
// -1 = no fit node of that class).  Scores are < 2^31 and chunks <= 4095 rows (host checks).
// Sweep lane l reads workgroups [l*MAXB, l*MAXB+MAXB): name-rank order is lane-major, so the
// matches above a workgroup are one wave prefix sum away.
#include "ksim_common.h"
#include "ksim_wave.h"

namespace {

constexpr int GR = KSIM_MAX_RCLASS;                  // granules per workgroup per slot
constexpr int MAXB = 4;                              // workgroups per sweep lane (grid <= 256)
constexpr uint64_t SPIN_LIMIT_TICKS = 200000000ull;  // s_memrealtime ticks at 100 MHz = 2 s

typedef __attribute__((address_space(1))) uint64_t gu64;

__device__ __forceinline__ void store_granule(uint64_t* g, uint64_t v) {
  __hip_atomic_store((gu64*)g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t load_granule(const uint64_t* g) {
  return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t gtag(uint64_t v) { return (uint32_t)(v >> 56); }
__device__ __forceinline__ int32_t gfit(uint64_t v) { return (int32_t)((v >> 44) & 0xFFF); }
__device__ __forceinline__ int32_t gcnt(uint64_t v) { return (int32_t)((v >> 32) & 0xFFF); }
__device__ __forceinline__ int32_t gscore(uint64_t v) { return (int32_t)(uint32_t)v; }

#ifdef KSIM_STAMPS
#define STAMP(k)                                         \
  do {                                                   \
    if (blockIdx.x == 0 && tid == 0) {                   \
      const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
      c.dbg[k] += t_ - t_prev;                          \
      t_prev = t_;                                      \
    }                                                    \
  } while (0)
#else
#define STAMP(k) \
  do {           \
  } while (0)
#endif

struct PDecision {
  int32_t mode;  // 0 none fit, 1 single fit, 2 select among winners, -1 abort
  int32_t blk;   // owner workgroup of the selected node
  int32_t rank;  // rank from the top (largest name rank) inside that workgroup
  uint32_t winners;
  int32_t row;   // owner only: committed row
  int32_t pad;
  int32_t M[KSIM_MAX_RCLASS];
};

struct Rows {  // LDS image of the owned rows (SoA)
  int64_t *ac, *am, *rc, *rm, *zc, *zm;
  int32_t *allowed, *count;
  uint32_t* fl;
};

__device__ __forceinline__ Rows carve(char* smem, int rows) {
  Rows r;
  int64_t* p = reinterpret_cast<int64_t*>(smem);
  r.ac = p; r.am = p + rows; r.rc = p + 2 * rows; r.rm = p + 3 * rows; r.zc = p + 4 * rows; r.zm = p + 5 * rows;
  int32_t* q = reinterpret_cast<int32_t*>(p + 6 * rows);
  r.allowed = q; r.count = q + rows;
  r.fl = reinterpret_cast<uint32_t*>(q + 2 * rows);
  return r;
}

// Commit of the columns that stay in HBM (gpu, ephemeral, scalars, ports) and of the
// over-commit bits (node_info.go:318-341, utils.go:45-60).  Single thread of the owner.
__device__ __forceinline__ uint32_t commit_side(const KsimCtx& c, const ksim_pod& P, int64_t w, uint32_t fl) {
  const int64_t g = c.req_gpu[w] + P.add_gpu;
  const int64_t e = c.req_eph[w] + P.add_eph;
  c.req_gpu[w] = g;
  c.req_eph[w] = e;
  fl &= ~(KSIM_N_GPU_OVER | KSIM_N_EPH_OVER);
  if (c.alloc_gpu[w] < g) fl |= KSIM_N_GPU_OVER;
  if (c.alloc_eph[w] < e) fl |= KSIM_N_EPH_OVER;
  for (int32_t s = 0; s < P.scalar_cnt; ++s) {
    const ksim_scalar_req q = c.pod_scalars[P.scalar_off + s];
    c.req_scalar[(int64_t)q.col * c.n + w] += q.add;
  }
  for (int32_t k = 0; k < P.port_cnt; ++k) {
    const uint64_t key = c.pod_ports[P.port_off + k];
    const int32_t cnt = c.port_count[w];
    bool dup = false;
    for (int32_t s = 0; s < cnt; ++s)
      if (c.ports[(int64_t)s * c.n + w] == key) { dup = true; break; }
    if (dup) continue;
    if (cnt >= c.port_slots) { atomicOr(c.err, 1); continue; }
    c.ports[(int64_t)cnt * c.n + w] = key;
    c.port_count[w] = cnt + 1;
  }
  return fl;
}

// Total score of reduce class q once the per-class maxima over the filtered set are known
// (NormalizeReduce, priorities/reduce.go:29-64; weighted sum generic_scheduler.go:632-639).
__device__ __forceinline__ int64_t class_total(const KsimCtx& c, const ksim_pod& P, int q, int k2, int64_t base,
                                               int64_t mxT, int64_t mxA) {
  uint64_t t = (uint64_t)base;
  if (c.w[KSIM_W_TAINT_TOLERATION])
    t += (uint64_t)c.w[KSIM_W_TAINT_TOLERATION] *
         (uint64_t)ksim_norm(c.tt_val[(int64_t)P.cls * KSIM_MAX_RCLASS + q / k2], mxT, true);
  if (c.w[KSIM_W_NODE_AFFINITY])
    t += (uint64_t)c.w[KSIM_W_NODE_AFFINITY] *
         (uint64_t)ksim_norm(c.na_val[(int64_t)P.cls * KSIM_MAX_RCLASS + q % k2], mxA, false);
  return (int64_t)t;
}

// Per-lane evaluation state of one pod over this lane's NPT rows.
template <int NPT>
struct Eval {
  bool fit[NPT];
  int32_t sc[NPT];
  int8_t cl[NPT];
  uint32_t rm[NPT];
};

struct PodInfo {
  int k1, k2, K;
};

__device__ __forceinline__ PodInfo pod_info(const KsimCtx& c, const ksim_pod& P) {
  PodInfo I;
  I.k1 = (c.w[KSIM_W_TAINT_TOLERATION] != 0) ? c.n_tt[P.cls] : 1;
  I.k2 = (c.w[KSIM_W_NODE_AFFINITY] != 0) ? c.n_na[P.cls] : 1;
  I.K = I.k1 * I.k2;
  return I;
}

__device__ __forceinline__ void eval_row(const KsimCtx& c, const Rows& R, const ksim_pod& P, const PodInfo& I,
                                         int64_t lo, int64_t j, bool& fit, int32_t& sc, int8_t& cl, uint32_t& rm) {
  const int64_t i = lo + j;
  KsimRow r;
  r.ac = R.ac[j]; r.am = R.am[j]; r.rc = R.rc[j]; r.rm = R.rm[j]; r.zc = R.zc[j]; r.zm = R.zm[j];
  r.allowed = R.allowed[j]; r.count = R.count[j]; r.fl = R.fl[j];
  const uint32_t m = ksim_predicates(c, P, i, r);
  fit = (m == 0);
  rm = m;
  sc = (int32_t)ksim_map_score(c, P, r);
  cl = (int8_t)((I.K > 1) ? ksim_rclass(c, P, i, I.k1, I.k2) : 0);
}

}  // namespace

template <int BS, int NPT>
__global__ __launch_bounds__(BS) void ksim_persistent_kernel(KsimCtx c, uint64_t* granules) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NW = BS / 64;
  __shared__ int32_t s_mx[NW][KSIM_MAX_RCLASS];
  __shared__ int32_t s_cnt[NW][KSIM_MAX_RCLASS];
  __shared__ int32_t s_fit[NW];
  __shared__ uint64_t s_gran[KSIM_MAX_RCLASS];  // next partial to publish (payload, no tag)
  __shared__ uint64_t s_ball[NPT][NW];
  __shared__ int32_t s_hist[KSIM_NREASONS];
  __shared__ int32_t s_M[KSIM_MAX_RCLASS];
  __shared__ int32_t s_C[KSIM_MAX_RCLASS];
  __shared__ PDecision D;

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int G = gridDim.x;
  const int64_t chunk = c.chunk;
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = (lo + chunk < c.n) ? lo + chunk : c.n;
  const int64_t nrows = hi - lo;
  Rows R = carve(smem, (int)chunk);

  for (int64_t j = tid; j < nrows; j += BS) {  // stage the owned rows into LDS
    const int64_t i = lo + j;
    R.ac[j] = c.alloc_cpu[i]; R.am[j] = c.alloc_mem[i];
    R.rc[j] = c.req_cpu[i]; R.rm[j] = c.req_mem[i];
    R.zc[j] = c.nz_cpu[i]; R.zm[j] = c.nz_mem[i];
    R.allowed[j] = c.allowed_pods[i]; R.count[j] = c.pod_count[i]; R.fl[j] = c.flags[i];
  }
  uint64_t counter = *c.counter;  // replicated genericScheduler.lastNodeIndex
  __syncthreads();

  // evaluate all owned rows for pod Q into E
  auto eval_all = [&](const ksim_pod& Q, const PodInfo& I, Eval<NPT>& E) {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int64_t j = (int64_t)k * BS + tid;
      E.fit[k] = false; E.sc[k] = -1; E.cl[k] = 0; E.rm[k] = 0;
      if (j < nrows) eval_row(c, R, Q, I, lo, j, E.fit[k], E.sc[k], E.cl[k], E.rm[k]);
    }
  };
  // block partial of E → s_gran (every thread calls; ends synchronised)
  auto reduce = [&](const Eval<NPT>& E, int K) {
    int32_t nf = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) nf += __popcll(__ballot(E.fit[k]));
    if (lane == 0) s_fit[wv] = nf;
    for (int q = 0; q < K; ++q) {
      int32_t v = -1;
#pragma unroll
      for (int k = 0; k < NPT; ++k)
        if (E.fit[k] && E.cl[k] == q && E.sc[k] > v) v = E.sc[k];
      const int32_t wm = ksimw::max_i32(v);
      int32_t n = 0;
#pragma unroll
      for (int k = 0; k < NPT; ++k) n += __popcll(__ballot(E.fit[k] && E.cl[k] == q && E.sc[k] == wm));
      if (lane == 0) { s_mx[wv][q] = wm; s_cnt[wv][q] = (wm < 0) ? 0 : n; }
    }
    __syncthreads();
    if (wv == 0 && lane < K) {
      int32_t m = -1, n = 0, f = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        f += s_fit[w];
        const int32_t cw = s_cnt[w][lane];
        if (cw == 0) continue;
        if (s_mx[w][lane] > m) { m = s_mx[w][lane]; n = cw; }
        else if (s_mx[w][lane] == m) n += cw;
      }
      s_gran[lane] = (lane == 0 ? ((uint64_t)f << 44) : 0) | ((uint64_t)n << 32) | (uint64_t)(uint32_t)m;
    }
    __syncthreads();
  };

  ksim_pod P = c.pods[c.first];
  PodInfo IP = pod_info(c, P);
  Eval<NPT> A, B;
  eval_all(P, IP, A);
  reduce(A, IP.K);
  ksim_pod Pn = c.pods[c.first + 1 < c.end ? c.first + 1 : c.first];
#ifdef KSIM_STAMPS
  uint64_t t_prev = __builtin_amdgcn_s_memtime();
#endif

  for (int64_t pod = c.first; pod < c.end; ++pod) {
    const int K = IP.K;
    const uint64_t tag = (uint64_t)((pod - c.first + 1) & 0xFF);
    uint64_t* slot = granules + (pod & 1) * (int64_t)G * GR;

    // ---------------- a. publish the partial of pod ----------------
    if (wv == 0 && lane < K) store_granule(slot + (int64_t)blockIdx.x * GR + lane, (tag << 56) | s_gran[lane]);
    STAMP(1);

    // ---------------- b. speculative evaluation of pod + 1 ----------------
    const bool has_next = pod + 1 < c.end;
    const ksim_pod Q = Pn;
    const PodInfo IQ = pod_info(c, Q);
    if (has_next) {
      Pn = c.pods[pod + 2 < c.end ? pod + 2 : pod + 1];
      eval_all(Q, IQ, B);
      reduce(B, IQ.K);
    }
    STAMP(0);

    // ---------------- c. sweep the partials of pod, decide ----------------
    if (wv == 0) {
      uint64_t g[MAXB];
      bool ok = false;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        bool mine = true;
#pragma unroll
        for (int j = 0; j < MAXB; ++j) {
          const int b = lane * MAXB + j;
          g[j] = 0;
          if (b < G) {
            g[j] = load_granule(slot + (int64_t)b * GR);
            mine &= gtag(g[j]) == tag;
          }
        }
#ifdef KSIM_STAMPS
        if (blockIdx.x == 0 && tid == 0) c.dbg[8] += 1;
#endif
        if (__all(mine)) { ok = true; break; }
        if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_LIMIT_TICKS) break;
        __builtin_amdgcn_s_sleep(1);
      }
      STAMP(2);
      ok = __all(ok);
      int32_t F = 0, M0 = -1, C0 = 0;
      if (ok) {
        int32_t f = 0, m = -1, n = 0;
#pragma unroll
        for (int j = 0; j < MAXB; ++j) {
          f += gfit(g[j]);
          const int32_t cnt = gcnt(g[j]), s = gscore(g[j]);
          if (cnt == 0) continue;
          if (s > m) { m = s; n = cnt; }
          else if (s == m) n += cnt;
        }
        F = ksimw::sum_i32(f);
        M0 = ksimw::max_i32(n ? m : -1);
        C0 = ksimw::sum_i32((n && m == M0) ? n : 0);
      }
      if (ok && K > 1) {  // further reduce classes (TaintToleration x NodeAffinity)
        if (lane == 0) { s_M[0] = M0; s_C[0] = C0; }
        for (int q = 1; q < K; ++q) {
          int32_t mm = -1, nn = 0;
          for (int j = 0; j < MAXB; ++j) {
            const int b = lane * MAXB + j;
            if (b >= G) break;
            uint64_t v = 0;
            const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
              v = load_granule(slot + (int64_t)b * GR + q);
              if (gtag(v) == tag) break;
              if (__builtin_amdgcn_s_memrealtime() - t1 > SPIN_LIMIT_TICKS) { ok = false; break; }
            }
            const int32_t cnt = gcnt(v), s = gscore(v);
            if (cnt == 0) continue;
            if (s > mm) { mm = s; nn = cnt; }
            else if (s == mm) nn += cnt;
          }
          const int32_t Mq = ksimw::max_i32(nn ? mm : -1);
          const int32_t Cq = ksimw::sum_i32((nn && mm == Mq) ? nn : 0);
          if (lane == 0) { s_M[q] = Mq; s_C[q] = Cq; }
        }
        ok = __all(ok);
      }
      if (!ok) {
        if (lane == 0) { D.mode = -1; atomicOr(c.err, 4); }
      } else if (F == 0) {
        if (lane == 0) D.mode = 0;
      } else {
        int mode = 1;
        uint32_t win = 1;
        int64_t ix = 0;
        if (F > 1) {  // generic_scheduler.go:153-156: a single fit skips selectHost
          mode = 2;
          int64_t C = C0;
          if (K > 1) {
            int64_t mxT = 0, mxA = 0;
            for (int q = 0; q < K; ++q) {
              if (s_C[q] == 0) continue;
              const int64_t tv = c.tt_val[(int64_t)P.cls * KSIM_MAX_RCLASS + q / IP.k2];
              const int64_t av = c.na_val[(int64_t)P.cls * KSIM_MAX_RCLASS + q % IP.k2];
              mxT = tv > mxT ? tv : mxT;
              mxA = av > mxA ? av : mxA;
            }
            int64_t best = INT64_MIN;
            for (int q = 0; q < K; ++q)
              if (s_C[q]) {
                const int64_t t = class_total(c, P, q, IP.k2, s_M[q], mxT, mxA);
                best = t > best ? t : best;
              }
            win = 0;
            C = 0;
            for (int q = 0; q < K; ++q)
              if (s_C[q] && class_total(c, P, q, IP.k2, s_M[q], mxT, mxA) == best) { win |= 1u << q; C += s_C[q]; }
          }
          ix = (int64_t)(counter % (uint64_t)C);  // generic_scheduler.go:192-195
          counter += 1;
        }
        // ---- locate the workgroup holding the ix-th match counted from the top ----
        int32_t bm[MAXB];
        int32_t tot = 0;
#pragma unroll
        for (int j = 0; j < MAXB; ++j) {
          const int b = lane * MAXB + j;
          int32_t m = 0;
          if (b < G) {
            if (mode == 1) {
              m = gfit(g[j]);
            } else {
              if ((win & 1u) && gcnt(g[j]) && gscore(g[j]) == M0) m += gcnt(g[j]);
              for (int q = 1; q < K; ++q) {
                if (!((win >> q) & 1u)) continue;
                const uint64_t v = load_granule(slot + (int64_t)b * GR + q);
                if (gcnt(v) && gscore(v) == s_M[q]) m += gcnt(v);
              }
            }
          }
          bm[j] = m;
          tot += m;
        }
        const int32_t pre = ksimw::prefix_incl_i32(tot);
        const int32_t total = __builtin_amdgcn_readlane(pre, 63);
        const int64_t above = (int64_t)(total - pre);  // matches in workgroups of higher lanes
        const bool hit = tot > 0 && ix >= above && ix < above + tot;
        if (hit) {
          int64_t r = ix - above;
          int found = -1;
#pragma unroll
          for (int j = MAXB - 1; j >= 0; --j) {
            if (found < 0) {
              if (r < bm[j]) found = lane * MAXB + j;
              else r -= bm[j];
            }
          }
          D.mode = found < 0 ? -1 : mode;
          D.blk = found;
          D.rank = (int32_t)r;
          D.winners = win;
          D.M[0] = M0;
          if (found < 0) atomicOr(c.err, 2);
        }
        if (K > 1 && lane > 0 && lane < K) D.M[lane] = s_M[lane];
        if (__ballot(hit) == 0 && lane == 0) { D.mode = -1; atomicOr(c.err, 2); }
      }
    }
    STAMP(3);
    __syncthreads();
    const int mode = D.mode;
    if (mode < 0) break;  // uniform: every workgroup reaches the same verdict

    if (mode == 0) {  // FitError: every workgroup adds its reasons; workgroup 0 records it
      if (c.collect && c.out_reasons) {
        if (tid < KSIM_NREASONS) s_hist[tid] = 0;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < NPT; ++k)
          for (int r = 0; r < KSIM_NREASONS; ++r) {
            const int32_t n = __popcll(__ballot((A.rm[k] >> r) & 1u));
            if (lane == 0 && n) atomicAdd(&s_hist[r], n);
          }
        __syncthreads();
        if (tid < KSIM_NREASONS && s_hist[tid]) atomicAdd(&c.out_reasons[pod * KSIM_NREASONS + tid], s_hist[tid]);
      }
      if (blockIdx.x == 0 && tid == 0) c.out_node[pod] = -1;
    } else if (D.blk == (int)blockIdx.x) {
      // ---------------- d. owner: exact node, commit, fix the speculative partial ----------
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        bool match = A.fit[k];
        if (mode == 2) match = A.fit[k] && ((D.winners >> A.cl[k]) & 1u) && A.sc[k] == D.M[A.cl[k]];
        const uint64_t bal = __ballot(match);
        if (lane == 0) s_ball[k][wv] = bal;
      }
      __syncthreads();
      if (tid == 0) {
        int32_t r = D.rank;
        int32_t j = -1;
        for (int k = NPT - 1; k >= 0 && j < 0; --k) {
          for (int w = NW - 1; w >= 0; --w) {
            uint64_t m = s_ball[k][w];
            const int nb = __popcll(m);
            if (r >= nb) { r -= nb; continue; }
            for (int t = 0; t < r; ++t) m &= ~(1ull << (63 - __clzll(m)));
            j = k * BS + w * 64 + (63 - __clzll(m));
            break;
          }
        }
        D.row = j;
        if (j < 0) {
          atomicOr(c.err, 2);
          c.out_node[pod] = -1;
        } else {
          const int64_t w = lo + j;
          R.rc[j] += P.add_cpu;
          R.rm[j] += P.add_mem;
          R.zc[j] += P.nz_cpu;
          R.zm[j] += P.nz_mem;
          R.count[j] += 1;
          if (P.add_gpu | P.add_eph | P.scalar_cnt | P.port_cnt) R.fl[j] = commit_side(c, P, w, R.fl[j]);
          c.out_node[pod] = (int32_t)w;
        }
      }
      __syncthreads();
      const int32_t j = D.row;
      if (has_next && j >= 0) {  // only row j changed: re-evaluate it for pod + 1, re-reduce
        if (j % BS == tid) {
#pragma unroll
          for (int k = 0; k < NPT; ++k)
            if (k == j / BS) eval_row(c, R, Q, IQ, lo, j, B.fit[k], B.sc[k], B.cl[k], B.rm[k]);
        }
        reduce(B, IQ.K);
      }
    }
    STAMP(4);
    // ---------------- e. pod + 1 becomes current ----------------
    A = B;
    P = Q;
    IP = IQ;
  }

  // the table is authoritative in HBM between calls: write the owned rows back
  __syncthreads();
  for (int64_t j = tid; j < nrows; j += BS) {
    const int64_t i = lo + j;
    c.req_cpu[i] = R.rc[j]; c.req_mem[i] = R.rm[j];
    c.nz_cpu[i] = R.zc[j]; c.nz_mem[i] = R.zm[j];
    c.pod_count[i] = R.count[j]; c.flags[i] = R.fl[j];
  }
  if (blockIdx.x == 0 && tid == 0) {
    *c.counter = counter;
    *c.cursor = c.end;
  }
}

// Checks the DPP wave helpers against plain lane loops (diagnostic, tests/ only).
__global__ void ksim_wave_selftest_kernel(int32_t* out) {
  const int lane = threadIdx.x;
  const int32_t v = (int32_t)((lane * 7919 + 13) % 97) - 40 + (blockIdx.x * 11);
  out[(blockIdx.x * 3 + 0) * 64 + lane] = ksimw::max_i32(v);
  out[(blockIdx.x * 3 + 1) * 64 + lane] = ksimw::sum_i32(v);
  out[(blockIdx.x * 3 + 2) * 64 + lane] = ksimw::prefix_incl_i32(v);
}

// ---------------------------------------------------------------------------------------
static constexpr int ROW_BYTES = 60;
static constexpr int LDS_BUDGET = 96 * 1024;

static int num_cus() {
  int dev = 0;
  hipDeviceProp_t p;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return 0;
  return p.multiProcessorCount;
}

// One workgroup per CU (<= 256) so every workgroup is resident — the protocol spins on every
// other workgroup — and chunk = ceil(n / grid) rows per workgroup held in LDS.
extern "C" int ksim_persistent_config(int64_t n, int* grid, int* lds_rows) {
  int g = num_cus();
  if (g <= 0 || n <= 0) return 0;
  if (g > 64 * MAXB) g = 64 * MAXB;
  if (n < (int64_t)g * 64) g = (int)((n + 63) / 64);  // >= 64 rows per workgroup
  if (g < 1) g = 1;
  const int64_t chunk = (n + g - 1) / g;
  if (chunk * ROW_BYTES > LDS_BUDGET || chunk > 4095) return 0;  // does not fit: launch mode
  *grid = g;
  *lds_rows = (int)chunk;
  return 1;
}

extern "C" size_t ksim_persistent_granule_bytes(int grid) { return (size_t)2 * grid * GR * sizeof(uint64_t); }

extern "C" hipError_t ksim_launch_persistent(const KsimCtx* c, uint64_t* granules, int grid, int lds_rows,
                                             hipStream_t s) {
  const size_t lds = (size_t)lds_rows * 64;
#define KSIM_PL(BS, NPT) \
  hipLaunchKernelGGL((ksim_persistent_kernel<BS, NPT>), dim3(grid), dim3(BS), lds, s, *c, granules)
  if (lds_rows <= 512) KSIM_PL(512, 1);
  else if (lds_rows <= 1024) KSIM_PL(512, 2);
  else if (lds_rows <= 2048) KSIM_PL(512, 4);
  else KSIM_PL(512, 8);
#undef KSIM_PL
  return hipGetLastError();
}

extern "C" int ksim_selftest(void) {
  int32_t* d = nullptr;
  const int nb = 4;
  if (hipMalloc(&d, nb * 3 * 64 * sizeof(int32_t)) != hipSuccess) return -1;
  hipLaunchKernelGGL(ksim_wave_selftest_kernel, dim3(nb), dim3(64), 0, 0, d);
  int32_t h[nb * 3 * 64];
  int bad = -1;
  if (hipDeviceSynchronize() == hipSuccess &&
      hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) == hipSuccess) {
    bad = 0;
    for (int b = 0; b < nb; ++b) {
      int32_t v[64], mx = INT32_MIN, sum = 0, pre = 0;
      for (int l = 0; l < 64; ++l) {
        v[l] = (int32_t)((l * 7919 + 13) % 97) - 40 + b * 11;
        mx = v[l] > mx ? v[l] : mx;
        sum += v[l];
      }
      for (int l = 0; l < 64; ++l) {
        pre += v[l];
        bad += h[(b * 3 + 0) * 64 + l] != mx;
        bad += h[(b * 3 + 1) * 64 + l] != sum;
        bad += h[(b * 3 + 2) * 64 + l] != pre;
      }
    }
  }
  (void)hipFree(d);
  return bad;
}
