// ksim_kernels.hip — gfx950 kernels of the per-pod scheduling cycle.
//
// Launch mode (KSIM_MODE_LAUNCH): one launch of ksim_scan_kernel per pod.  Every block
// evaluates a contiguous, name-ordered chunk of nodes (one node per lane per step),
// reduces it to a per-reduce-class (max map score, count at max) + fit count (+ reason
// histogram) partial, publishes it, and takes an arrival ticket.  The last block to
// arrive acquires, combines all partials into the global decision (findNodesThatFit
// → PrioritizeNodes → selectHost, core/generic_scheduler.go:112-198), locates the
// selected node by walking block counts from the highest name rank down, picks the exact
// node from that block's published candidate masks (KSIM_PM_*: per wave and reduce class, the
// ballot of nodes at the wave's maximum), commits the pod (NodeInfo.AddPod) and advances
// the device-side pod cursor.  Launches are replayed from a hipGraph, so per-pod host
// work is zero and no PCIe traffic happens between pods.
#include "ksim_common.h"
#include "ksim_wave.h"

namespace {

// wave reductions on the DPP helpers (row shifts / broadcasts, no LDS permute)
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) { return ksimw::max_i64(v); }
__device__ __forceinline__ int32_t wave_sum_i32(int32_t v) { return ksimw::sum_i32(v); }

// inclusive prefix sum over the 256-thread block (4 waves)
__device__ __forceinline__ int64_t block_incl_scan(int64_t v, int64_t* s_w) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  if (lane == 63) s_w[wv] = v;
  __syncthreads();
  int64_t add = 0;
  for (int k = 0; k < wv; ++k) add += s_w[k];
  __syncthreads();
  return v + add;
}

// cross-device exchange words (fine-grained buffers written by peers over xGMI)
__device__ __forceinline__ void lx_store(uint64_t* g, uint64_t v) {
  __hip_atomic_store(g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t lx_load(const uint64_t* g) {
  return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Decision {
  int64_t pod;
  int32_t K, K2;
  int32_t fitTotal;
  int32_t mode;      // 0: none fit, 1: single fit, 2: select among winners
  uint32_t winners;  // reduce classes whose total equals the max
  int64_t M[KSIM_MAX_RCLASS];
  int64_t ix;        // rank from the top (largest name rank)
  int64_t blk;       // selected block
  int64_t rank;      // rank within the selected block from the top
  int64_t node;
};

}  // namespace

// InterPodAffinityPriority inputs of one pod: whether it reads the priority and the min / max
// of its raw per-node sums over the fit nodes (written by ksim_ipa_pass_kernel just before).
// Same for SelectorSpread: the pod's counted pair and the pass-A maxima.
struct IpaNorm {
  bool on;
  int64_t mn, mx, w;
  int32_t sp;          // SelectorSpread counted pair, -1: off
  bool hz;             // haveZones
  int64_t sw, smx, szmx;
  // the auxiliary priority (KsimAff::aux_*): aon = the pod reads it, ap = its counted pair (-1: no
  // counts, no pass A), and the pass-A words
  bool aon, ahz;
  int32_t ap, akind;
  int64_t aw, amx, atot, azmx;
};

__device__ __forceinline__ IpaNorm ipa_norm(const KsimCtx& c, const ksim_pod& P) {
  IpaNorm z{false, 0, 0, 0, -1, false, 0, 0, 0, false, false, -1, 0, 0, 0, 0, 0};
  if (!c.aff || c.no_prio) return z;
  if (c.w[KSIM_W_INTERPOD_AFFINITY] != 0 && ksim_interpod_prio_work(*c.aff, P)) {
    z.on = true;
    z.mn = c.aff->mm[0];
    z.mx = c.aff->mm[1];
    z.w = c.w[KSIM_W_INTERPOD_AFFINITY];
  }
  if (c.w[KSIM_W_SELECTOR_SPREAD] != 0 && (z.sp = ksim_spread_pair(*c.aff, P)) >= 0) {
    z.sw = c.w[KSIM_W_SELECTOR_SPREAD];
    z.smx = c.aff->mm[2];
    z.hz = c.aff->mm[3] != 0;
    z.szmx = c.aff->mm[4];
  }
  const KsimAff& A = *c.aff;
  if (A.aux_pair && A.aux_w != 0) {
    z.ap = ksim_aux_pair(A, P);
    z.akind = A.aux_kind;
    // a pod without a pair: ServiceAntiAffinity still scores by the node's label (no counts);
    // the spread reduce of zero counts is MaxPriority everywhere (a constant, left out)
    z.aon = z.ap >= 0 || z.akind == KSIM_AUX_SERVICE_ANTI;
    z.aw = A.aux_w;
    if (z.ap >= 0) {
      z.amx = A.mm[5];
      z.atot = A.mm[6];
      z.ahz = A.mm[7] != 0;
      z.azmx = A.mm[8];
    }
  }
  return z;
}

// The auxiliary priority's weighted score of fit node i (count cnt, domain d): ap < 0 reads no count.
__device__ __forceinline__ uint64_t aux_add(const KsimAff& A, const IpaNorm& z, int64_t cnt, int32_t d) {
  const int64_t ds = (z.ap >= 0 && d >= 0) ? A.aread[d] : 0;
  return (uint64_t)z.aw * (uint64_t)ksim_aux_score(z.akind, z.ap >= 0 ? cnt : 0, d, ds, z.amx, z.atot, z.ahz, z.azmx);
}

// Evaluate one node for the scan: fit, map score (+ the normalised InterPodAffinity score),
// reduce class, reason mask.
template <bool COLLECT>
__device__ __forceinline__ void eval_one(const KsimCtx& c, const ksim_pod& P, int64_t i, int k1, int k2,
                                         const IpaNorm& ipa, bool& fit, int64_t& score, int& cls, uint32_t& rmask) {
  fit = false; score = 0; cls = 0; rmask = 0;
  if (i >= c.n) return;
  const KsimRow r = ksim_load_row(c, i);
  const uint32_t m = ksim_predicates(c, P, i, r);
  fit = (m == 0);
  if (COLLECT) rmask = m;
  score = ksim_map_score(c, P, r);
  if (ipa.on && fit)
    score = (int64_t)((uint64_t)score +
                      (uint64_t)ipa.w * (uint64_t)ksim_interpod_score(ksim_interpod_raw_body(*c.aff, P, i), ipa.mn, ipa.mx));
  if (ipa.sp >= 0 && fit) {
    const KsimAff& A = *c.aff;
    const int32_t z = A.zone_key >= 0 ? ksim_dom(A, A.zone_key, i) : -1;
    const int64_t v = ksim_spread_score(A.cnt[A.pair_off[ipa.sp] + i], ipa.smx, ipa.hz, z, z >= 0 ? A.zread[z] : 0, ipa.szmx);
    score = (int64_t)((uint64_t)score + (uint64_t)ipa.sw * (uint64_t)v);
  }
  if (ipa.aon && fit) {
    const KsimAff& A = *c.aff;
    const int64_t cnt = ipa.ap >= 0 ? A.cnt[A.pair_off[ipa.ap] + i] : 0;
    score = (int64_t)((uint64_t)score + aux_add(A, ipa, cnt, ksim_dom(A, A.aux_key, i)));
  }
  cls = (k1 * k2 > 1) ? ksim_rclass(c, P, i, k1, k2) : 0;
}

// The resident per-pod kernel's rows between messages: each thread keeps the 60-byte rows of the
// nodes it evaluates (and their label / taint set ids) in registers for the kernel's lifetime — the
// block that owns a node is the only one that reads or commits it, and the committing block reloads
// the row after each commit — so an evaluation starts without a dependent load chain.
template <int NPT>
struct KsimRowCache {
  KsimRow r[NPT];
  int32_t ls[NPT], ts[NPT];
};

// The pod class's table entries for one node, loaded together up front (the ids are in registers):
// one round trip instead of a set id load followed by a table load per predicate.
struct KsimPrefAcc {
  const KsimCtx& c;
  bool sel, tok, nok;
  int ttc, nac;
  __device__ __forceinline__ bool sel_ok(const ksim_pod&, int64_t) const { return sel; }
  __device__ __forceinline__ bool taint_ok(const ksim_pod&, int64_t) const { return tok; }
  __device__ __forceinline__ bool noexec_ok(const ksim_pod&, int64_t) const { return nok; }
  __device__ __forceinline__ bool port_conflict(int64_t i, uint64_t want) const { return ksim_port_conflict(c, i, want); }
  __device__ __forceinline__ uint64_t want(const ksim_pod& P, int32_t k) const { return ksim_pod_port(c, P, k); }
  __device__ __forceinline__ int tt_class(const ksim_pod&, int64_t) const { return ttc; }
  __device__ __forceinline__ int na_class(const ksim_pod&, int64_t) const { return nac; }
};

// eval_one over a cached row (the resident kernel): the same predicates, priorities and classes.
template <bool COLLECT>
__device__ __forceinline__ void eval_cached(const KsimCtx& c, const ksim_pod& P, int64_t i, const KsimRow& r, int32_t ls,
                                            int32_t ts, int k1, int k2, bool& fit, int64_t& score, int& cls, uint32_t& rmask) {
  fit = false; score = 0; cls = 0; rmask = 0;
  if (i >= c.n) return;
  KsimPrefAcc a{c, true, true, true, 0, 0};
  const int64_t cl = P.cls;
  if (P.flags & KSIM_POD_NEED_SELECTOR) a.sel = ksim_bit(c.sel_ok, cl, c.lwords, ls);
  if (P.flags & KSIM_POD_NEED_TAINTS) {
    a.tok = ksim_bit(c.taint_ok, cl, c.twords, ts);
    a.nok = ksim_bit(c.noexec_ok, cl, c.twords, ts);
  }
  if (k1 > 1) a.ttc = c.tt_class[cl * c.n_taint_sets + ts];
  if (k2 > 1) a.nac = c.na_class[cl * c.n_label_sets + ls];
  const uint32_t m = ksim_predicates_a<KsimPrefAcc, true, true>(c, P, i, r, a);
  fit = (m == 0);
  if (COLLECT) rmask = m;
  score = ksim_map_score(c, P, r);
  cls = (k1 * k2 > 1) ? ksim_rclass_a(P, i, k1, k2, a) : 0;
}

// Pass A of an InterPodAffinityPriority / SelectorSpread pod, over the fit nodes: min / max of the
// raw InterPodAffinity sums with 0 folded in as the reference's accumulators start there
// (interpod_affinity.go:129-131, 218-226); SelectorSpread's maxCountByNodeName, haveZones and
// countsByZone (selector_spreading.go:125-145, zone sums by atomics).  Every block reduces its
// chunk to a partial; the last block to arrive combines them into aff->mm, publishes the zone sums
// (zread) with their maximum, zeroes zsum for the next pod and re-arms the ticket.  Returns true
// in that block.  Run either as its own launch before the scan (ksim_ipa_pass_kernel) or fused
// into the scan behind a grid barrier (KsimCtx::fuse_a).
#define KSIM_PASS_ZONES 512
#define KSIM_PASS_V 7   // pass-A words combined per wave (s_v rows)
template <int NPT>
__device__ __forceinline__ bool passa_reduce(const KsimCtx& c, int64_t pod, bool ipa, int32_t sp, int32_t ap,
                                             const bool (&fit)[NPT],
                                             const int64_t (&raw)[NPT], const int64_t (&cnt)[NPT],
                                             const int32_t (&zz)[NPT], const int64_t (&acnt)[NPT],
                                             const int32_t (&azz)[NPT], int64_t (*s_v)[KSIM_WAVES],
                                             unsigned long long* s_z, int* s_last) {
  const KsimAff& A = *c.aff;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const bool zlocal = A.n_zone <= KSIM_PASS_ZONES;
  if (sp >= 0 && zlocal) {
    for (int z = tid; z < A.n_zone; z += KSIM_BLOCK) s_z[z] = 0;
    __syncthreads();
  }
  int64_t mn = 0, mx = 0, smx = 0, hz = 0, amx = 0, atot = 0, ahz = 0;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    if (!fit[k]) continue;
    if (ipa) {
      mn = raw[k] < mn ? raw[k] : mn;
      mx = raw[k] > mx ? raw[k] : mx;
    }
    if (sp >= 0) {
      const int64_t v = cnt[k];
      smx = v > smx ? v : smx;
      const int32_t z = zz[k];
      if (z >= 0) {
        hz = 1;
        if (v) {
          if (zlocal) atomicAdd(&s_z[z], (unsigned long long)v);
          else atomicAdd(reinterpret_cast<unsigned long long*>(&A.zsum[z]), (unsigned long long)v);
        }
      }
    }
    if (ap >= 0) {  // the auxiliary priority: max, sum, haveZones and per-domain sums (global adds)
      const int64_t v = acnt[k];
      amx = v > amx ? v : amx;
      atot += v;
      if (azz[k] >= 0) {
        ahz = 1;
        if (v) atomicAdd(reinterpret_cast<unsigned long long*>(&A.asum[azz[k]]), (unsigned long long)v);
      }
    }
  }
  if (sp >= 0 && zlocal) {  // one global add per (block, zone) with a count
    __syncthreads();
    for (int z = tid; z < A.n_zone; z += KSIM_BLOCK)
      if (s_z[z]) atomicAdd(reinterpret_cast<unsigned long long*>(&A.zsum[z]), s_z[z]);
  }
  // every wave's zone atomics have landed before the barrier that precedes this block's ticket
  // (thread 0's release fence covers its own wave only)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  auto combine = [&]() {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const int64_t a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
      const int64_t d = __shfl_xor(smx, o, 64), e = __shfl_xor(hz, o, 64);
      mn = a < mn ? a : mn;
      mx = b > mx ? b : mx;
      smx = d > smx ? d : smx;
      hz = e > hz ? e : hz;
      if (ap >= 0) {
        const int64_t f = __shfl_xor(amx, o, 64), g = __shfl_xor(atot, o, 64), q = __shfl_xor(ahz, o, 64);
        amx = f > amx ? f : amx;
        atot += g;
        ahz = q > ahz ? q : ahz;
      }
    }
    if (lane == 0) {
      s_v[0][wv] = mn; s_v[1][wv] = mx; s_v[2][wv] = smx; s_v[3][wv] = hz;
      s_v[4][wv] = amx; s_v[5][wv] = atot; s_v[6][wv] = ahz;
    }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < KSIM_WAVES; ++w) {
        mn = s_v[0][w] < mn ? s_v[0][w] : mn;
        mx = s_v[1][w] > mx ? s_v[1][w] : mx;
        smx = s_v[2][w] > smx ? s_v[2][w] : smx;
        hz = s_v[3][w] > hz ? s_v[3][w] : hz;
        amx = s_v[4][w] > amx ? s_v[4][w] : amx;
        atot += s_v[5][w];
        ahz = s_v[6][w] > ahz ? s_v[6][w] : ahz;
      }
    }
  };
  combine();
  if (tid == 0) {
    int64_t* pp = A.part + KSIM_AFF_PART * (int64_t)blockIdx.x;
    pp[0] = mn; pp[1] = mx; pp[2] = smx; pp[3] = hz;
    pp[4] = amx; pp[5] = atot; pp[6] = ahz;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(A.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_last = (old == gridDim.x - 1);
  }
  __syncthreads();
  if (!*s_last) return false;
  if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  mn = 0; mx = 0; smx = 0; hz = 0; amx = 0; atot = 0; ahz = 0;
  for (int b = tid; b < (int)gridDim.x; b += KSIM_BLOCK) {
    const int64_t* pp = A.part + KSIM_AFF_PART * (int64_t)b;
    mn = pp[0] < mn ? pp[0] : mn;
    mx = pp[1] > mx ? pp[1] : mx;
    smx = pp[2] > smx ? pp[2] : smx;
    hz = pp[3] > hz ? pp[3] : hz;
    if (ap >= 0) {
      amx = pp[4] > amx ? pp[4] : amx;
      atot += pp[5];
      ahz = pp[6] > ahz ? pp[6] : ahz;
    }
  }
  __syncthreads();
  combine();
  __syncthreads();
  int64_t r0 = mn, r1 = mx, r2 = smx, r3 = hz;  // valid in thread 0
  const int64_t r5 = amx, r6 = atot, r7 = ahz;
  // zone sums: publish for the scan, zero for the next pod, maximum (countsByZone, :139-143)
  int64_t zmx = 0, azm = 0;
  if (c.sh_world > 1) {
    // node-sharded (SURVEY.md §8e Phase A): this rank's pass-A words to every rank, the world's
    // min / max / max / haveZones and zone sums back, then (a pod with an auxiliary count) the
    // auxiliary priority's max / sum / haveZones and domain sums
    const int nz = sp >= 0 ? A.n_zone : 0;   // <= KSIM_PX_ZONES (host-checked)
    const int na = ap >= 0 ? A.n_adom : 0;   // <= KSIM_PX_ADOMS (host-checked)
    const int A0 = 4 + nz, W = A0 + (ap >= 0 ? 3 + na : 0), me = c.sh_rank;
    // word x's combine over the ranks: 0 = min, 1 = max, 2 = sum
    const int op = lane == 0 ? 0 : (lane < 4 ? 1 : (lane < A0 ? 2 : (lane == A0 || lane == A0 + 2 ? 1 : 2)));
    if (tid == 0) {
      s_v[0][0] = r0; s_v[1][0] = r1; s_v[2][0] = r2; s_v[3][0] = r3;
      s_v[4][0] = r5; s_v[5][0] = r6; s_v[6][0] = r7;
    }
    __syncthreads();
    int64_t* px = reinterpret_cast<int64_t*>(s_z);  // [KSIM_MAX_RANKS][KSIM_PX_REC] (the zone scratch is free now)
    if (wv == 0) {
      const uint64_t tag = (uint64_t)(1u + (uint32_t)((c.sh_tag0 + (uint64_t)(pod - c.first)) % 0xFFFFFFull)) << 40;
      const uint64_t vmask = (1ull << 40) - 1;
      const int slot = (int)(pod % KSIM_LX_SLOTS);
      uint64_t* const base0 = c.sh_peers[me] + (int64_t)KSIM_LX_SLOTS * KSIM_MAX_RANKS * KSIM_LX_REC;
      if (lane < W) {
        const int64_t v =
            lane < 4    ? s_v[lane][0]
            : lane < A0 ? (int64_t)__hip_atomic_load(&A.zsum[lane - 4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
            : lane < A0 + 3 ? s_v[4 + lane - A0][0]
                            : (int64_t)__hip_atomic_load(&A.asum[lane - A0 - 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        px[me * KSIM_PX_REC + lane] = v;
        for (int r = 0; r < c.sh_world; ++r)
          lx_store(c.sh_peers[r] + (int64_t)KSIM_LX_SLOTS * KSIM_MAX_RANKS * KSIM_LX_REC +
                       ((int64_t)slot * KSIM_MAX_RANKS + me) * KSIM_PX_REC + lane,
                   tag | ((uint64_t)(v + KSIM_LX_BIAS) & vmask));
      }
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      const uint64_t lim = pod == c.first ? c.sh_start_ticks : 200000000ull;  // 2 s at 100 MHz
      for (;;) {
        bool ready = true;
        for (int x = lane; x < c.sh_world * W; x += 64) {
          const int r = x / W, j = x % W;
          if (r == me) continue;
          const uint64_t v = lx_load(base0 + ((int64_t)slot * KSIM_MAX_RANKS + r) * KSIM_PX_REC + j);
          if ((v & ~vmask) != tag) { ready = false; continue; }
          px[r * KSIM_PX_REC + j] = (int64_t)(v & vmask) - KSIM_LX_BIAS;
        }
        if (__all(ready)) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > lim) {
          if (lane == 0) atomicOr(c.err, 4);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      // the world's words, then the zone / domain sums published and their maxima
      int64_t g = 0;
      if (lane < W) {
        g = px[lane];
        for (int r = 1; r < c.sh_world; ++r) {
          const int64_t v = px[r * KSIM_PX_REC + lane];
          g = op == 0 ? (v < g ? v : g) : (op == 1 ? (v > g ? v : g) : g + v);
        }
        if (lane >= 4 && lane < A0) {
          A.zread[lane - 4] = g;
          A.zsum[lane - 4] = 0;
        } else if (lane >= A0 + 3) {
          A.aread[lane - A0 - 3] = g;
          A.asum[lane - A0 - 3] = 0;
        }
      }
      const int64_t zm = wave_max_i64(lane >= 4 && lane < A0 ? g : 0);
      const int64_t am = wave_max_i64(lane >= A0 + 3 && lane < W ? g : 0);
      r0 = __shfl(g, 0, 64); r1 = __shfl(g, 1, 64); r2 = __shfl(g, 2, 64); r3 = __shfl(g, 3, 64);
      const int64_t g5 = __shfl(g, A0 & 63, 64), g6 = __shfl(g, (A0 + 1) & 63, 64), g7 = __shfl(g, (A0 + 2) & 63, 64);
      if (lane == 0) {
        A.mm[0] = r0 < 0 ? r0 : 0;  // (the accumulators start at 0: every rank's are <= 0 / >= 0 already)
        A.mm[1] = r1;
        A.mm[2] = r2;
        A.mm[3] = r3;
        A.mm[4] = zm;
        if (ap >= 0) {
          A.mm[5] = g5;
          A.mm[6] = g6;
          A.mm[7] = g7;
          A.mm[8] = am;
        }
        *A.ticket = 0;
      }
    }
    return true;
  }
  if (sp >= 0)
    for (int z = tid; z < A.n_zone; z += KSIM_BLOCK) {
      const int64_t v = __hip_atomic_load(&A.zsum[z], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      A.zread[z] = v;
      A.zsum[z] = 0;
      zmx = v > zmx ? v : zmx;
    }
  if (ap >= 0)
    for (int z = tid; z < A.n_adom; z += KSIM_BLOCK) {
      const int64_t v = __hip_atomic_load(&A.asum[z], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      A.aread[z] = v;
      A.asum[z] = 0;
      azm = v > azm ? v : azm;
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t a = __shfl_xor(zmx, o, 64), b = __shfl_xor(azm, o, 64);
    zmx = a > zmx ? a : zmx;
    azm = b > azm ? b : azm;
  }
  if (lane == 0) { s_v[0][wv] = zmx; s_v[1][wv] = azm; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < KSIM_WAVES; ++w) {
      zmx = s_v[0][w] > zmx ? s_v[0][w] : zmx;
      azm = s_v[1][w] > azm ? s_v[1][w] : azm;
    }
    A.mm[0] = r0;
    A.mm[1] = r1;
    A.mm[2] = r2;
    A.mm[3] = r3;
    A.mm[4] = zmx;
    A.mm[5] = r5;
    A.mm[6] = r6;
    A.mm[7] = r7;
    A.mm[8] = azm;
    *A.ticket = 0;
  }
  return true;
}

// Pass A as its own launch (pods that read neither priority exit at once, uniformly).
template <int NPT>
__global__ __launch_bounds__(KSIM_BLOCK) void ksim_ipa_pass_kernel(KsimCtx c) {
  __shared__ int64_t s_v[KSIM_PASS_V][KSIM_WAVES];
  __shared__ unsigned long long s_z[KSIM_PASS_ZONES];  // block-local zone sums (few zones: no global contention)
  __shared__ int s_last;
  const int64_t pod = c.one ? c.first : *c.cursor;
  if (pod >= c.end || !c.aff || c.no_prio) return;
  // node-sharded: a peer that never answered (err bit 4) ends the run for every later launch
  // (one read broadcast through LDS: the exit is uniform across the block's waves)
  if (c.sh_world > 1) {
    __shared__ int s_stop;
    if (threadIdx.x == 0) s_stop = __hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 4;
    __syncthreads();
    if (s_stop) return;
  }
  ksim_pod P;  // (a branch, not a pointer select: the pod stays in registers)
  if (c.one) P = c.one_pod;
  else P = c.pods[pod];
  const KsimAff& A = *c.aff;
  const bool ipa = c.w[KSIM_W_INTERPOD_AFFINITY] != 0 && ksim_interpod_prio_work(A, P);
  const int32_t sp = c.w[KSIM_W_SELECTOR_SPREAD] != 0 ? ksim_spread_pair(A, P) : -1;
  const int32_t ap = A.aux_w != 0 ? ksim_aux_pair(A, P) : -1;
  if (!ipa && sp < 0 && ap < 0) return;
  const int64_t base = (int64_t)blockIdx.x * c.chunk;
  bool fit[NPT];
  int64_t raw[NPT], cnt[NPT], acnt[NPT];
  int32_t zz[NPT], azz[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int64_t i = base + k * KSIM_BLOCK + threadIdx.x;
    fit[k] = false; raw[k] = 0; cnt[k] = 0; zz[k] = -1; acnt[k] = 0; azz[k] = -1;
    if (i >= c.n) continue;
    const KsimRow r = ksim_load_row(c, i);
    if (ksim_predicates(c, P, i, r) != 0) continue;
    fit[k] = true;
    if (ipa) raw[k] = ksim_interpod_raw_body(A, P, i);
    if (sp >= 0) {
      cnt[k] = A.cnt[A.pair_off[sp] + i];
      zz[k] = A.zone_key >= 0 ? ksim_dom(A, A.zone_key, i) : -1;
    }
    if (ap >= 0) {
      acnt[k] = A.cnt[A.pair_off[ap] + i];
      azz[k] = ksim_dom(A, A.aux_key, i);
    }
  }
  (void)passa_reduce<NPT>(c, pod, ipa, sp, ap, fit, raw, cnt, zz, acnt, azz, s_v, s_z, &s_last);
}

// diagnostic builds (make stamps): thread 0's cycles per scan phase, summed over blocks into
// dbg[48..58] (every block: 48 pod read, 49 evaluation, 50 candidate masks + statistics, 51 partial
// + ticket; the last block: 52 combine, 53 decide, 54 locate, 55 masks + pick, 56 commit,
// 57 results), dbg[60] blocks, dbg[61] last blocks; printed by ksim_destroy
#ifdef KSIM_STAMPS
#define SSTAMP(k)                                          \
  do {                                                     \
    if (tid == 0) {                                        \
      const uint64_t t_ = __builtin_amdgcn_s_memtime();   \
      st_acc[k] += t_ - ts_prev;                           \
      ts_prev = t_;                                        \
    }                                                      \
  } while (0)
// thread 0 adds its sums at the block's exit (no global atomic between the phases it times)
#define SFLUSH()                                                                                   \
  do {                                                                                             \
    if (tid == 0)                                                                                  \
      for (int k_ = 0; k_ < 10; ++k_)                                                              \
        if (st_acc[k_]) atomicAdd((unsigned long long*)&c.dbg[48 + k_], (unsigned long long)st_acc[k_]); \
  } while (0)
#else
#define SSTAMP(k) \
  do {            \
  } while (0)
#define SFLUSH() \
  do {           \
  } while (0)
#endif

template <int NPT, bool COLLECT>
__global__ __launch_bounds__(KSIM_BLOCK) void ksim_scan_kernel(KsimCtx c) {
  __shared__ int64_t s_mx[KSIM_WAVES][KSIM_MAX_RCLASS];
  __shared__ int32_t s_cnt[KSIM_WAVES][KSIM_MAX_RCLASS];
  __shared__ int32_t s_fit[KSIM_WAVES];
  __shared__ int32_t s_hist[KSIM_NREASONS];
  __shared__ int64_t s_scan[KSIM_WAVES];
  __shared__ uint64_t s_ball[NPT][KSIM_WAVES];
  __shared__ int s_last;
  __shared__ Decision D;
  __shared__ int64_t s_v[KSIM_PASS_V][KSIM_WAVES];     // fused pass A
  __shared__ unsigned long long s_z[KSIM_PASS_ZONES];
  __shared__ uint32_t s_gen;
  __shared__ int s_bail;
  __shared__ uint64_t s_ctr;
  __shared__ int64_t s_Mq[KSIM_MAX_RCLASS], s_tot[KSIM_MAX_RCLASS];
  __shared__ int32_t s_Cq[KSIM_MAX_RCLASS];
  __shared__ int64_t s_tv[KSIM_MAX_WIDE], s_av[KSIM_MAX_WIDE], s_ad[KSIM_MAX_WIDE];
  // wide pods (K > KSIM_MAX_RCLASS): per class the block's max and count, then the grid's, and the
  // winning classes
  __shared__ int64_t s_wm[KSIM_MAX_WIDE];
  __shared__ int32_t s_wc[KSIM_MAX_WIDE];
  __shared__ uint8_t s_ww[KSIM_MAX_WIDE];
  // node-sharded launch form: every rank's fit count and per-class (max, count)
  __shared__ int64_t s_rM[KSIM_MAX_RANKS][KSIM_MAX_RCLASS];
  __shared__ int32_t s_rC[KSIM_MAX_RANKS][KSIM_MAX_RCLASS];
  __shared__ int32_t s_rF[KSIM_MAX_RANKS];
  __shared__ int s_shok;
  // last block, single reduce class: every block's (fit, max, count) as combined, for the locate step
  constexpr int LOC_MAX = 1024;
  __shared__ int64_t s_bmx[LOC_MAX];
  __shared__ int32_t s_bcnt[LOC_MAX], s_bfit[LOC_MAX];
  static_assert(NPT <= KSIM_PM_NPT, "candidate masks hold KSIM_PM_NPT node slots per thread");

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#ifdef KSIM_STAMPS
  uint64_t ts_prev = __builtin_amdgcn_s_memtime();
  uint64_t st_acc[10] = {};
  if (tid == 0) atomicAdd((unsigned long long*)&c.dbg[60], 1ull);
#endif
  if (c.fuse_a) {
    // a fused barrier that timed out (err bit 64) left this run's tickets mid-pod: every later
    // launch of the graph exits at once (uniformly per block) and the host resumes unfused
    if (tid == 0) s_bail = (int)__hip_atomic_load(c.ticket + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (s_bail) return;
  }
  const int64_t pod = c.one ? c.first : *c.cursor;
  if (pod >= c.end) return;  // uniform: graph replay past the end of the queue
  // node-sharded: a peer that never answered (err bit 4) ends the run for every later launch
  // (one read broadcast through LDS: the exit is uniform across the block's waves)
  if (c.sh_world > 1) {
    if (tid == 0) s_bail = __hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 4;
    __syncthreads();
    if (s_bail) return;
  }
  ksim_pod P;  // (a branch, not a pointer select: the pod stays in registers)
  if (c.one) P = c.one_pod;
  else P = c.pods[pod];
  // per-pod launches carry the class's reduce-class counts in the descriptor (stage_pod)
  const int k1 = c.one ? P.reserved[0] : (c.w[KSIM_W_TAINT_TOLERATION] != 0) ? c.n_tt[P.cls] : 1;
  const int k2 = c.one ? P.reserved[1] : c.use_na ? c.n_na[P.cls] : 1;
  const int K = k1 * k2;
  const bool wide = K > KSIM_MAX_RCLASS;  // uniform: the wide decision (per-class arrays in LDS / global)
  // what the last block's decision reads, fetched now while the chunk is evaluated: the counter
  // (kernels of a stream run one after another, so its value is final) and the pod's per-class
  // TaintToleration / NodeAffinity values and NodePreferAvoidPods addends
  // (loaded into registers here, stored to LDS after the evaluation: the loads overlap it)
  uint64_t pre_ctr = 0;
  int64_t pre_tv = 0, pre_av = 0, pre_ad = 0;
  if (tid == 0) pre_ctr = *c.counter;
  if (tid < K) {
    pre_tv = c.tt_val[(int64_t)P.cls * c.val_w + tid / k2];
    pre_av = c.na_val[(int64_t)P.cls * c.val_w + tid % k2];
    pre_ad = c.na_add ? c.na_add[(int64_t)P.cls * c.val_w + tid % k2] : 0;
  }
  const int64_t base = (int64_t)blockIdx.x * c.chunk;
  IpaNorm ipa = ipa_norm(c, P);
  // fused pass A (KsimCtx::fuse_a, grid co-resident): this pod's pass-A reductions run over the
  // fit nodes evaluated here, behind one grid barrier (generation word ticket[1], read before
  // this block's pass-A ticket), and the normalised scores are added afterwards
  const bool fuse = c.fuse_a && (ipa.on || ipa.sp >= 0 || ipa.ap >= 0);
  IpaNorm ipa0 = ipa;
  if (fuse) {
    ipa0.on = false;
    ipa0.sp = -1;
    if (ipa.ap >= 0) ipa0.aon = false;
    if (tid == 0) {
      s_bail = 0;
      s_gen = __hip_atomic_load(c.ticket + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }

  if (COLLECT && tid < KSIM_NREASONS) s_hist[tid] = 0;
  SSTAMP(0);

  // ---------------- phase 1: evaluate this block's chunk ----------------
  bool fit[NPT];
  int64_t sc[NPT];
  int cl[NPT];
  uint32_t rm[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k)
    eval_one<COLLECT>(c, P, base + k * KSIM_BLOCK + tid, k1, k2, ipa0, fit[k], sc[k], cl[k], rm[k]);

  if (fuse) {
    const KsimAff& A = *c.aff;
    int64_t raw[NPT], cnt[NPT], acnt[NPT];
    int32_t zz[NPT], azz[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int64_t i = base + k * KSIM_BLOCK + tid;
      raw[k] = 0; cnt[k] = 0; zz[k] = -1; acnt[k] = 0; azz[k] = -1;
      if (!fit[k]) continue;
      if (ipa.on) raw[k] = ksim_interpod_raw_body(A, P, i);
      if (ipa.sp >= 0) {
        cnt[k] = A.cnt[A.pair_off[ipa.sp] + i];
        zz[k] = A.zone_key >= 0 ? ksim_dom(A, A.zone_key, i) : -1;
      }
      if (ipa.ap >= 0) {
        acnt[k] = A.cnt[A.pair_off[ipa.ap] + i];
        azz[k] = ksim_dom(A, A.aux_key, i);
      }
    }
    if (passa_reduce<NPT>(c, pod, ipa.on, ipa.sp, ipa.ap, fit, raw, cnt, zz, acnt, azz, s_v, s_z, &s_last)) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's zread stores
      __syncthreads();
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(c.ticket + 1, s_gen + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      if (tid == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(c.ticket + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == s_gen) {
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t0 > c.barrier_ticks) {  // 2 s: blocks not co-resident
            atomicOr(c.err, 64);
            __hip_atomic_store(c.ticket + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_bail = 1;
            break;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (s_bail) return;
    }
    ipa = ipa_norm(c, P);  // the combined maxima
#pragma unroll
    for (int k = 0; k < NPT; ++k) {  // eval_one's additions (modular sums: any order)
      if (!fit[k]) continue;
      if (ipa.on)
        sc[k] = (int64_t)((uint64_t)sc[k] + (uint64_t)ipa.w * (uint64_t)ksim_interpod_score(raw[k], ipa.mn, ipa.mx));
      if (ipa.sp >= 0) {
        const int64_t v = ksim_spread_score(cnt[k], ipa.smx, ipa.hz, zz[k], zz[k] >= 0 ? A.zread[zz[k]] : 0, ipa.szmx);
        sc[k] = (int64_t)((uint64_t)sc[k] + (uint64_t)ipa.sw * (uint64_t)v);
      }
      if (ipa.ap >= 0) sc[k] = (int64_t)((uint64_t)sc[k] + aux_add(A, ipa, acnt[k], azz[k]));
    }
  }

  SSTAMP(1);
  if (tid == 0) s_ctr = pre_ctr;
  if (tid < K) {
    s_tv[tid] = pre_tv;
    s_av[tid] = pre_av;
    s_ad[tid] = pre_ad;
  }
  // candidate masks: write-through (sc1) stores, drained by every storing wave before the barrier
  // that precedes the ticket, read back with sc1 loads by the last block
  uint64_t* pm = c.pmask + (int64_t)blockIdx.x * KSIM_PM_STRIDE;
  int32_t nfit = 0;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const uint64_t b = __ballot(fit[k]);
    nfit += __popcll(b);
    if (lane == 0) __hip_atomic_store(&pm[KSIM_PM_MASK(KSIM_MAX_RCLASS, k, wv)], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (lane == 0) s_fit[wv] = nfit;

  if (wide) {
    // per class: the block's max map score among its fit nodes (LDS max), then the count at it
    for (int q = tid; q < K; q += KSIM_BLOCK) { s_wm[q] = INT64_MIN; s_wc[q] = 0; }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NPT; ++k)
      if (fit[k]) __hip_atomic_fetch_max(&s_wm[cl[k]], sc[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NPT; ++k)
      if (fit[k] && sc[k] == s_wm[cl[k]]) atomicAdd(&s_wc[cl[k]], 1);
    __syncthreads();
    for (int q = tid; q < K; q += KSIM_BLOCK) {
      c.wmx[(int64_t)blockIdx.x * KSIM_MAX_WIDE + q] = s_wm[q];
      c.wcnt[(int64_t)blockIdx.x * KSIM_MAX_WIDE + q] = s_wc[q];
    }
  }
#pragma unroll
  for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
    if (q >= K || wide) break;
    int64_t v = INT64_MIN;
#pragma unroll
    for (int k = 0; k < NPT; ++k)
      if (fit[k] && cl[k] == q && sc[k] > v) v = sc[k];
    const int64_t wm = wave_max_i64(v);
    int32_t n = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const uint64_t b = __ballot(fit[k] && cl[k] == q && sc[k] == wm);
      n += __popcll(b);
      if (lane == 0) __hip_atomic_store(&pm[KSIM_PM_MASK(q, k, wv)], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_mx[wv][q] = wm;
      s_cnt[wv][q] = (wm == INT64_MIN) ? 0 : n;
      __hip_atomic_store(reinterpret_cast<int64_t*>(&pm[KSIM_PM_MX(q, wv)]), wm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (COLLECT) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      if (__ballot(rm[k] != 0)) {
        for (int r = 0; r < KSIM_NREASONS; ++r) {
          const int32_t n = __popcll(__ballot((rm[k] >> r) & 1u));
          if (lane == 0 && n) atomicAdd(&s_hist[r], n);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  SSTAMP(2);

  // ---------------- publish the partial, take a ticket ----------------
  if (tid == 0) {
    KsimPartial* p = &c.partials[blockIdx.x];
    int32_t f = 0;
    for (int w = 0; w < KSIM_WAVES; ++w) f += s_fit[w];
    p->fit = f;
    for (int q = 0; q < (wide ? 0 : K); ++q) {
      int64_t m = INT64_MIN;
      int32_t n = 0;
      for (int w = 0; w < KSIM_WAVES; ++w) {
        if (s_cnt[w][q] == 0) continue;
        if (s_mx[w][q] > m) { m = s_mx[w][q]; n = s_cnt[w][q]; }
        else if (s_mx[w][q] == m) n += s_cnt[w][q];
      }
      p->mx[q] = m;
      p->cnt[q] = n;
    }
    if (COLLECT)
      for (int r = 0; r < KSIM_NREASONS; ++r) p->hist[r] = s_hist[r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(c.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (old == gridDim.x - 1);
  }
  __syncthreads();
  SSTAMP(3);
  if (!s_last) {
    SFLUSH();
    return;
  }

  // ---------------- last block: the global decision ----------------
#ifdef KSIM_STAMPS
  if (tid == 0) atomicAdd((unsigned long long*)&c.dbg[61], 1ull);
#endif
  if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int G = gridDim.x;
  // combine partials: each thread a strided set of blocks
  int64_t lm[KSIM_MAX_RCLASS];
  int32_t ln[KSIM_MAX_RCLASS];
  int32_t lf = 0;
#pragma unroll
  for (int q = 0; q < KSIM_MAX_RCLASS; ++q) { lm[q] = INT64_MIN; ln[q] = 0; }
  const bool loc_lds = K == 1 && G <= LOC_MAX;
  for (int b = tid; b < G; b += KSIM_BLOCK) {
    const KsimPartial* p = &c.partials[b];
    lf += p->fit;
    if (loc_lds) {
      s_bfit[b] = p->fit;
      s_bcnt[b] = p->cnt[0];
      s_bmx[b] = p->mx[0];
    }
#pragma unroll
    for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
      if (q >= K || wide) break;
      const int32_t n = p->cnt[q];
      if (n == 0) continue;
      const int64_t m = p->mx[q];
      if (m > lm[q]) { lm[q] = m; ln[q] = n; }
      else if (m == lm[q]) ln[q] += n;
    }
  }
  const int32_t wf = wave_sum_i32(lf);
  if (lane == 0) s_fit[wv] = wf;
#pragma unroll
  for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
    if (q >= K || wide) break;
    const int64_t wm = wave_max_i64(ln[q] ? lm[q] : INT64_MIN);
    const int32_t wn = wave_sum_i32((ln[q] && lm[q] == wm) ? ln[q] : 0);
    if (lane == 0) { s_mx[wv][q] = wm; s_cnt[wv][q] = wn; }
  }
  __syncthreads();
  SSTAMP(4);

  if (c.sh_world > 1) {
    // ---- node-sharded: the world's decision inputs (SURVEY.md §8e Phase A) ----
    const int me = c.sh_rank, W = 1 + 2 * K;
    if (tid == 0) {
      int32_t F = 0;
      for (int w = 0; w < KSIM_WAVES; ++w) F += s_fit[w];
      s_rF[me] = F;
      for (int q = 0; q < K; ++q) {
        int64_t m = INT64_MIN;
        int32_t n = 0;
        for (int w = 0; w < KSIM_WAVES; ++w) {
          if (s_cnt[w][q] == 0) continue;
          if (s_mx[w][q] > m) { m = s_mx[w][q]; n = s_cnt[w][q]; }
          else if (s_mx[w][q] == m) n += s_cnt[w][q];
        }
        s_rM[me][q] = m;
        s_rC[me][q] = n;
      }
      s_shok = 1;
    }
    __syncthreads();
    if (wv == 0) {
      const uint64_t tag = (uint64_t)(1u + (uint32_t)((c.sh_tag0 + (uint64_t)(pod - c.first)) % 0xFFFFFFull)) << 40;
      const int slot = (int)(pod % KSIM_LX_SLOTS);
      const uint64_t vmask = (1ull << 40) - 1;
      auto word = [&](int j) -> uint64_t {  // this rank's word j: F, then (max + bias, count) per class
        if (j == 0) return (uint64_t)(uint32_t)s_rF[me];
        const int q = (j - 1) >> 1;
        if ((j - 1) & 1) return (uint64_t)(uint32_t)s_rC[me][q];
        return s_rC[me][q] ? (uint64_t)(s_rM[me][q] + KSIM_LX_BIAS) & vmask : 0ull;
      };
      for (int x = lane; x < c.sh_world * W; x += 64) {
        const int r = x / W, j = x % W;
        lx_store(c.sh_peers[r] + ((int64_t)slot * KSIM_MAX_RANKS + me) * KSIM_LX_REC + j, tag | word(j));
      }
      const uint64_t* mine = c.sh_peers[me] + (int64_t)slot * KSIM_MAX_RANKS * KSIM_LX_REC;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      const uint64_t lim = pod == c.first ? c.sh_start_ticks : 200000000ull;  // 2 s at 100 MHz
      for (;;) {
        bool ready = true;
        for (int x = lane; x < c.sh_world * W; x += 64) {
          const int r = x / W, j = x % W;
          if (r == me) continue;
          const uint64_t v = lx_load(mine + (int64_t)r * KSIM_LX_REC + j);
          if ((v & ~vmask) != tag) { ready = false; continue; }
          const uint64_t val = v & vmask;
          if (j == 0) s_rF[r] = (int32_t)val;
          else if ((j - 1) & 1) s_rC[r][(j - 1) >> 1] = (int32_t)val;
          else s_rM[r][(j - 1) >> 1] = (int64_t)val - KSIM_LX_BIAS;
        }
        if (__all(ready)) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > lim) {
          if (lane == 0) { atomicOr(c.err, 4); s_shok = 0; }
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    if (!s_shok) {  // a peer never answered: the run ends here (the host reports it)
      if (tid == 0) { c.out_node[pod] = -1; *c.ticket = 0; }
      return;
    }
    // the world's inputs in the slots the decision below reads (wave 0's; the other waves' cleared)
    if (tid == 0) {
      int32_t F = 0;
      for (int r = 0; r < c.sh_world; ++r) F += s_rF[r];
      s_fit[0] = F;
      for (int w = 1; w < KSIM_WAVES; ++w) s_fit[w] = 0;
      for (int q = 0; q < K; ++q) {
        int64_t m = INT64_MIN;
        int32_t n = 0;
        for (int r = 0; r < c.sh_world; ++r) {
          if (s_rC[r][q] == 0) continue;
          if (s_rM[r][q] > m) { m = s_rM[r][q]; n = s_rC[r][q]; }
          else if (s_rM[r][q] == m) n += s_rC[r][q];
        }
        s_mx[0][q] = m;
        s_cnt[0][q] = n;
        for (int w = 1; w < KSIM_WAVES; ++w) s_cnt[w][q] = 0;
      }
    }
    __syncthreads();
  }

  if (wide) {
    // the grid's max and count per class (thread q), the NormalizeReduce maxima over the present
    // classes, each class's total and the winners (generic_scheduler.go:632-639, reduce.go:29-64)
    int64_t tq = INT64_MIN, mT = 0, mA = 0;
    for (int q = tid; q < K; q += KSIM_BLOCK) {
      int64_t m = INT64_MIN;
      int32_t n = 0;
      for (int b = 0; b < G; ++b) {
        const int32_t cb = c.wcnt[(int64_t)b * KSIM_MAX_WIDE + q];
        if (!cb) continue;
        const int64_t mb = c.wmx[(int64_t)b * KSIM_MAX_WIDE + q];
        if (mb > m) { m = mb; n = cb; }
        else if (mb == m) n += cb;
      }
      s_wm[q] = m;
      s_wc[q] = n;
      if (n) {
        if (k1 > 1 || c.w[KSIM_W_TAINT_TOLERATION]) mT = s_tv[q] > mT ? s_tv[q] : mT;
        if (k2 > 1 || c.w[KSIM_W_NODE_AFFINITY]) mA = s_av[q] > mA ? s_av[q] : mA;
      }
    }
    mT = wave_max_i64(mT);
    mA = wave_max_i64(mA);
    if (lane == 0) { s_v[0][wv] = mT; s_v[1][wv] = mA; }
    __syncthreads();
    mT = 0; mA = 0;
    for (int w = 0; w < KSIM_WAVES; ++w) {
      mT = s_v[0][w] > mT ? s_v[0][w] : mT;
      mA = s_v[1][w] > mA ? s_v[1][w] : mA;
    }
    for (int q = tid; q < K; q += KSIM_BLOCK) {
      if (!s_wc[q]) continue;
      uint64_t t = (uint64_t)s_wm[q];
      if (c.w[KSIM_W_TAINT_TOLERATION]) t += (uint64_t)c.w[KSIM_W_TAINT_TOLERATION] * (uint64_t)ksim_norm(s_tv[q], mT, true);
      if (c.w[KSIM_W_NODE_AFFINITY]) t += (uint64_t)c.w[KSIM_W_NODE_AFFINITY] * (uint64_t)ksim_norm(s_av[q], mA, false);
      t += (uint64_t)s_ad[q];
      tq = (int64_t)t > tq ? (int64_t)t : tq;
    }
    const int64_t best_w = wave_max_i64(tq);
    __syncthreads();  // s_v reused
    if (lane == 0) s_v[0][wv] = best_w;
    __syncthreads();
    int64_t best = INT64_MIN;
    for (int w = 0; w < KSIM_WAVES; ++w) best = s_v[0][w] > best ? s_v[0][w] : best;
    int64_t cw = 0;
    for (int q = tid; q < K; q += KSIM_BLOCK) {
      bool win = false;
      if (s_wc[q]) {
        uint64_t t = (uint64_t)s_wm[q];
        if (c.w[KSIM_W_TAINT_TOLERATION]) t += (uint64_t)c.w[KSIM_W_TAINT_TOLERATION] * (uint64_t)ksim_norm(s_tv[q], mT, true);
        if (c.w[KSIM_W_NODE_AFFINITY]) t += (uint64_t)c.w[KSIM_W_NODE_AFFINITY] * (uint64_t)ksim_norm(s_av[q], mA, false);
        t += (uint64_t)s_ad[q];
        win = (int64_t)t == best;
      }
      s_ww[q] = win ? 1 : 0;
      if (win) cw += s_wc[q];
    }
    __syncthreads();  // s_v reused
    const int32_t cws = wave_sum_i32((int32_t)cw);
    if (lane == 0) s_cnt[wv][0] = cws;
    __syncthreads();
  }

  if (tid == 0) {
    D.pod = pod;
    D.K = K;
    D.K2 = k2;
    int32_t F = 0;
    for (int w = 0; w < KSIM_WAVES; ++w) F += s_fit[w];
    D.fitTotal = F;
    D.node = -1;
    D.blk = -1;
    D.rank = 0;
    if (F == 0) {
      D.mode = 0;
    } else if (F == 1) {  // generic_scheduler.go:153-156: no selectHost, no counter bump
      D.mode = 1;
      D.ix = 0;
    } else if (wide) {  // the winners and their count from the wide combine above
      D.mode = 2;
      int64_t C = 0;
      for (int w = 0; w < KSIM_WAVES; ++w) C += s_cnt[w][0];
      D.winners = 0;
      const uint64_t li = s_ctr;  // generic_scheduler.go:192-195
      D.ix = ((li >> 32) == 0 && C < ((int64_t)1 << 32)) ? (int64_t)((uint32_t)li % (uint32_t)C) : (int64_t)(li % (uint64_t)C);
      *c.counter = li + 1;
      s_ctr = li + 1;
    } else if (K == 1) {  // one reduce class: it wins, its count at the maximum is C
      D.mode = 2;
      int64_t m = INT64_MIN;
      int32_t n = 0;
      for (int w = 0; w < KSIM_WAVES; ++w) {
        const int32_t cw = s_cnt[w][0];
        const int64_t mw = s_mx[w][0];
        if (cw == 0) continue;
        if (mw > m) { m = mw; n = cw; }
        else if (mw == m) n += cw;
      }
      D.winners = 1u;
      D.M[0] = m;
      const uint64_t li = s_ctr;  // generic_scheduler.go:192-195
      const int64_t C = n;
      D.ix = ((li >> 32) == 0 && C < ((int64_t)1 << 32)) ? (int64_t)((uint32_t)li % (uint32_t)C) : (int64_t)(li % (uint64_t)C);
      *c.counter = li + 1;
      s_ctr = li + 1;
    } else {
      D.mode = 2;
      int64_t* const Mq = s_Mq;  // per-class arrays in LDS: private arrays indexed by a run-time
      int32_t* const Cq = s_Cq;  // class would live in scratch memory
      int64_t* const tot = s_tot;
      for (int q = 0; q < K; ++q) {
        int64_t m = INT64_MIN;
        int32_t n = 0;
        for (int w = 0; w < KSIM_WAVES; ++w) {
          if (s_cnt[w][q] == 0) continue;
          if (s_mx[w][q] > m) { m = s_mx[w][q]; n = s_cnt[w][q]; }
          else if (s_mx[w][q] == m) n += s_cnt[w][q];
        }
        Mq[q] = m;
        Cq[q] = n;
      }
      // reduce priorities over the filtered set (NormalizeReduce)
      int64_t mxT = 0, mxA = 0;
      for (int q = 0; q < K; ++q) {
        if (Cq[q] == 0) continue;
        const int64_t tv = s_tv[q];
        const int64_t av = s_av[q];
        if (k1 > 1 || c.w[KSIM_W_TAINT_TOLERATION]) mxT = tv > mxT ? tv : mxT;
        if (k2 > 1 || c.w[KSIM_W_NODE_AFFINITY]) mxA = av > mxA ? av : mxA;
      }
      int64_t best = INT64_MIN;
      for (int q = 0; q < K; ++q) {
        if (Cq[q] == 0) continue;
        uint64_t t = (uint64_t)Mq[q];
        if (c.w[KSIM_W_TAINT_TOLERATION]) t += (uint64_t)c.w[KSIM_W_TAINT_TOLERATION] * (uint64_t)ksim_norm(s_tv[q], mxT, true);
        if (c.w[KSIM_W_NODE_AFFINITY]) t += (uint64_t)c.w[KSIM_W_NODE_AFFINITY] * (uint64_t)ksim_norm(s_av[q], mxA, false);
        t += (uint64_t)s_ad[q];  // NodePreferAvoidPods (0 without the addends)
        tot[q] = (int64_t)t;
        if (tot[q] > best) best = tot[q];
      }
      uint32_t win = 0;
      int64_t C = 0;
      for (int q = 0; q < K; ++q)
        if (Cq[q] && tot[q] == best) { win |= 1u << q; C += Cq[q]; }
      D.winners = win;
      for (int q = 0; q < K; ++q) D.M[q] = Mq[q];
      const uint64_t li = s_ctr;                // generic_scheduler.go:192-195
      D.ix = ((li >> 32) == 0 && C < ((int64_t)1 << 32)) ? (int64_t)((uint32_t)li % (uint32_t)C) : (int64_t)(li % (uint64_t)C);
      *c.counter = li + 1;
      s_ctr = li + 1;
    }
  }
  __syncthreads();
  SSTAMP(5);

  if (c.sh_world > 1 && D.mode != 0) {
    // selectHost's ix-th node from the top: ranks hold ascending name-rank shards, so the ranks above
    // this one come first; this rank holds it when ix falls among its own matches
    if (tid == 0) {
      int64_t above = 0, here = 0;
      for (int r = 0; r < c.sh_world; ++r) {
        int64_t m = 0;
        if (D.mode == 1) {
          m = s_rF[r];
        } else {
          for (int q = 0; q < K; ++q)
            if (((D.winners >> q) & 1u) && s_rC[r][q] && s_rM[r][q] == D.M[q]) m += s_rC[r][q];
        }
        if (r > c.sh_rank) above += m;
        else if (r == c.sh_rank) here = m;
      }
      const int64_t ixl = D.ix - above;
      if (ixl >= 0 && ixl < here) D.ix = ixl;
      else D.mode = 3;  // another rank holds the node
    }
    __syncthreads();
  }

  if (D.mode == 3) {
    if (tid == 0) D.node = -2;  // another rank's node (read by thread 0 below)
  } else if (D.mode == 0) {
    if (COLLECT && c.out_reasons) {
      for (int r = 0; r < KSIM_NREASONS; ++r) {
        int32_t v = 0;
        for (int b = tid; b < G; b += KSIM_BLOCK) v += c.partials[b].hist[r];
        v = wave_sum_i32(v);
        if (lane == 0) s_cnt[wv][0] = v;
        __syncthreads();
        if (tid == 0) c.out_reasons[pod * KSIM_NREASONS + r] = s_cnt[0][0] + s_cnt[1][0] + s_cnt[2][0] + s_cnt[3][0];
        __syncthreads();
      }
    }
  } else {
    // ---- locate the block holding the ix-th match counted from the top ----
    const int64_t per = (G + KSIM_BLOCK - 1) / KSIM_BLOCK;
    const int tr = KSIM_BLOCK - 1 - tid;  // reversed: thread 0 owns the highest blocks
    const int64_t b0 = (int64_t)tr * per, b1 = (b0 + per < G) ? b0 + per : G;
    // matches in block b (the partials kept in LDS by the combine step when K == 1)
    auto matches = [&](int64_t b) -> int64_t {
      if (loc_lds) return D.mode == 1 ? s_bfit[b] : ((s_bcnt[b] && s_bmx[b] == D.M[0]) ? s_bcnt[b] : 0);
      const KsimPartial* p = &c.partials[b];
      if (D.mode == 1) return p->fit;
      if (wide) {
        int64_t cw = 0;
        for (int q = 0; q < K; ++q) {
          if (!s_ww[q]) continue;
          const int32_t n = c.wcnt[b * KSIM_MAX_WIDE + q];
          if (n && c.wmx[b * KSIM_MAX_WIDE + q] == s_wm[q]) cw += n;
        }
        return cw;
      }
      int64_t cb = 0;
      for (int q = 0; q < K; ++q)
        if (((D.winners >> q) & 1u) && p->cnt[q] && p->mx[q] == D.M[q]) cb += p->cnt[q];
      return cb;
    };
    int64_t s = 0;
    for (int64_t b = b0; b < b1; ++b) s += matches(b);
    const int64_t incl = block_incl_scan(s, s_scan);
    const int64_t above = incl - s;
    if (s > 0 && D.ix >= above && D.ix < incl) {
      int64_t r = D.ix - above;
      for (int64_t b = b1 - 1; b >= b0; --b) {
        const int64_t cb = matches(b);
        if (r < cb) { D.blk = b; D.rank = r; break; }
        r -= cb;
      }
    }
    __syncthreads();
    SSTAMP(6);
    if (D.blk < 0) {  // inconsistent partials: must never happen
      if (tid == 0) { atomicOr(c.err, 2); c.out_node[pod] = -1; *c.cursor = pod + 1; *c.ticket = 0; }
      return;
    }
    // ---- the selected block's candidate masks (no re-evaluation), pick the exact node ----
    const int64_t bb = D.blk * c.chunk;
    if (wide && D.mode == 2) {
      // no per-class masks: the selected block's nodes evaluated again, with the final maxima
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        bool f;
        int64_t sk;
        int qk;
        uint32_t rk;
        eval_one<false>(c, P, bb + k * KSIM_BLOCK + tid, k1, k2, ipa, f, sk, qk, rk);
        const uint64_t b = __ballot(f && s_ww[qk] && sk == s_wm[qk]);
        if (lane == 0) s_ball[k][wv] = b;
      }
    } else if (tid < NPT * KSIM_WAVES) {
      const int k = tid / KSIM_WAVES, w = tid % KSIM_WAVES;
      uint64_t* pb = c.pmask + D.blk * KSIM_PM_STRIDE;
      uint64_t m = 0;
      if (D.mode == 1) {
        m = __hip_atomic_load(&pb[KSIM_PM_MASK(KSIM_MAX_RCLASS, k, w)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        for (int q = 0; q < K; ++q) {
          if (!((D.winners >> q) & 1u)) continue;
          const int64_t wm = __hip_atomic_load(reinterpret_cast<int64_t*>(&pb[KSIM_PM_MX(q, w)]), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
          if (wm == D.M[q])
            m |= __hip_atomic_load(&pb[KSIM_PM_MASK(q, k, w)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      s_ball[k][w] = m;
    }
    __syncthreads();
    if (tid == 0) {
      int64_t r = D.rank;
      int64_t node = -1;
      for (int k = NPT - 1; k >= 0 && node < 0; --k) {
        for (int w = KSIM_WAVES - 1; w >= 0; --w) {
          uint64_t m = s_ball[k][w];
          const int n = __popcll(m);
          if (r >= n) { r -= n; continue; }
          for (int64_t j = 0; j < r; ++j) m &= ~(1ull << (63 - __clzll(m)));
          node = bb + (int64_t)k * KSIM_BLOCK + w * 64 + (63 - __clzll(m));
          break;
        }
      }
      if (node < 0) atomicOr(c.err, 2);  // inconsistent partials: must never happen
      D.node = node;
    }
    __syncthreads();
    SSTAMP(7);
    // commit: the row and volumes in thread 0, the affinity counts across wave 1 meanwhile
    if (D.node >= 0 && !c.no_commit) {
      if (wv == 0) {
        const int32_t st = ksim_commit_wave(c, P, D.node, lane);
        if (tid == 0) {
          if (ksim_is_vol_pod(c, P)) ksim_vol_commit_body(*c.vol, P, D.node, 1, c.err);
          if (c.out_fit) c.out_fit[1] |= st;
        }
      } else if (wv == 1 && ksim_is_aff_pod(c, P)) {
        if (lane == 0) ksim_svc_commit(*c.aff, P, D.node);  // reads the counts before this commit's adds
        ksim_aff_commit_body(*c.aff, P, D.node, 1, lane, 64);
      }
    }
  }
  if (c.out_fit) __syncthreads();  // (uniform) wave 1's affinity commit is done
  SSTAMP(8);
  if (tid == 0) {
    c.out_node[pod] = (int32_t)(c.sh_world > 1 && D.node >= 0 ? c.sh_base + D.node : D.node);
    if (c.out_fit) {  // per-pod drop-in: fit count, error word and lastNodeIndex into the result block
      c.out_fit[0] = D.fitTotal;
      c.out_fit[KSIM_RES_ERR - KSIM_RES_FIT] = __hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t ctr = s_ctr;
      c.out_fit[KSIM_RES_CTR - KSIM_RES_FIT] = (int32_t)(uint32_t)ctr;
      c.out_fit[KSIM_RES_CTR - KSIM_RES_FIT + 1] = (int32_t)(uint32_t)(ctr >> 32);
    }
    if (!c.one) *c.cursor = pod + 1;
    *c.ticket = 0;
  }
  SSTAMP(9);
  SFLUSH();
}

// ---------------------------------------------------------------------------------------
// The per-pod call on a cluster one workgroup covers (ksim_schedule_one, n <= 16 x 512): the
// same evaluation, pass A, decision and commit as ksim_scan_kernel, with every cross-node
// reduction in LDS — no partials, arrival ticket, candidate masks or second pass through global
// memory, so the launch is bounded by the evaluation's own load chains.  Pass A's zone sums stay
// in LDS (<= KSIM_PASS_ZONES zones, host-checked); the pod comes from the kernel arguments.
constexpr int ONE_BLOCK = 512;  // 2 waves per SIMD: 256 VGPRs for the NPT evaluations in flight
constexpr int ONE_WAVES = ONE_BLOCK / 64;

template <int NPT>
__global__ __launch_bounds__(ONE_BLOCK) void ksim_one_kernel(KsimCtx c) {
  __shared__ int64_t s_mx[ONE_WAVES][KSIM_MAX_RCLASS];
  __shared__ int32_t s_cnt[ONE_WAVES][KSIM_MAX_RCLASS];
  __shared__ int32_t s_fit[ONE_WAVES];
  __shared__ int32_t s_hist[KSIM_NREASONS];
  __shared__ int64_t s_v[7][ONE_WAVES];
  __shared__ unsigned long long s_z[KSIM_PASS_ZONES];
  __shared__ uint64_t s_bm[NPT][ONE_WAVES];
  __shared__ Decision D;
  __shared__ int64_t s_pa[9];  // pass A: min / max raw InterPodAffinity sum, max spread count, haveZones, zone max,
                               // the auxiliary priority's max count, summed count, haveZones, domain max
  __shared__ unsigned long long s_az[KSIM_PASS_ZONES];  // the auxiliary priority's domain sums (<= 512, host-checked)

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const ksim_pod P = c.one_pod;
  const int64_t pod = c.first;
  const int k1 = P.reserved[0], k2 = P.reserved[1];
  const int K = k1 * k2 <= KSIM_MAX_RCLASS ? k1 * k2 : KSIM_MAX_RCLASS;  // (the host never sends a wide pod here)
  // the decision's inputs, loaded while the nodes are evaluated (to LDS afterwards)
  __shared__ int64_t s_tv[KSIM_MAX_RCLASS], s_av[KSIM_MAX_RCLASS], s_ad[KSIM_MAX_RCLASS];
  uint64_t pre_ctr = 0;
  int64_t pre_tv = 0, pre_av = 0, pre_ad = 0;
  if (tid == 0) pre_ctr = *c.counter;
  if (tid < K) {
    pre_tv = c.tt_val[(int64_t)P.cls * c.val_w + tid / k2];
    pre_av = c.na_val[(int64_t)P.cls * c.val_w + tid % k2];
    pre_ad = c.na_add ? c.na_add[(int64_t)P.cls * c.val_w + tid % k2] : 0;
  }
  IpaNorm ipa = ipa_norm(c, P);  // which of pass A's priorities the pod reads (maxima below)
  IpaNorm ipa0 = ipa;
  ipa0.on = false;
  ipa0.sp = -1;
  ipa0.aon = false;
  const bool pass_a = ipa.on || ipa.sp >= 0 || ipa.aon;
  if (tid < KSIM_NREASONS) s_hist[tid] = 0;
  if (ipa.sp >= 0)
    for (int z = tid; z < c.aff->n_zone; z += ONE_BLOCK) s_z[z] = 0;
  if (ipa.ap >= 0)
    for (int z = tid; z < c.aff->n_adom; z += ONE_BLOCK) s_az[z] = 0;
  if (ipa.sp >= 0 || ipa.ap >= 0) __syncthreads();  // (uniform) the domain sums are zero before the atomics

  bool fit[NPT];
  int64_t sc[NPT];
  int cl[NPT];
  uint32_t rm[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) eval_one<true>(c, P, (int64_t)k * ONE_BLOCK + tid, k1, k2, ipa0, fit[k], sc[k], cl[k], rm[k]);

  if (pass_a) {  // (uniform) pass A over the fit nodes, reduced in LDS
    const KsimAff& A = *c.aff;
    int64_t raw[NPT], cnt[NPT];
    int32_t zz[NPT];
    int64_t mn = 0, mx = 0, smx = 0, hz = 0, amx = 0, atot = 0, ahz = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int64_t i = (int64_t)k * ONE_BLOCK + tid;
      raw[k] = 0; cnt[k] = 0; zz[k] = -1;
      if (!fit[k]) continue;
      if (ipa.on) {
        raw[k] = ksim_interpod_raw_body(A, P, i);
        mn = raw[k] < mn ? raw[k] : mn;
        mx = raw[k] > mx ? raw[k] : mx;
      }
      if (ipa.sp >= 0) {
        cnt[k] = A.cnt[A.pair_off[ipa.sp] + i];
        zz[k] = A.zone_key >= 0 ? ksim_dom(A, A.zone_key, i) : -1;
        smx = cnt[k] > smx ? cnt[k] : smx;
        if (zz[k] >= 0) {
          hz = 1;
          if (cnt[k]) atomicAdd(&s_z[zz[k]], (unsigned long long)cnt[k]);
        }
      }
      if (ipa.ap >= 0) {  // the auxiliary priority (passa_reduce's): max, sum, haveZones, domain sums
        const int64_t v = A.cnt[A.pair_off[ipa.ap] + i];
        const int32_t d = ksim_dom(A, A.aux_key, i);
        amx = v > amx ? v : amx;
        atot += v;
        if (d >= 0) {
          ahz = 1;
          if (v) atomicAdd(&s_az[d], (unsigned long long)v);
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const int64_t a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
      const int64_t d = __shfl_xor(smx, o, 64), e = __shfl_xor(hz, o, 64);
      mn = a < mn ? a : mn;
      mx = b > mx ? b : mx;
      smx = d > smx ? d : smx;
      hz = e > hz ? e : hz;
      if (ipa.ap >= 0) {
        const int64_t f = __shfl_xor(amx, o, 64), g = __shfl_xor(atot, o, 64), q = __shfl_xor(ahz, o, 64);
        amx = f > amx ? f : amx;
        atot += g;
        ahz = q > ahz ? q : ahz;
      }
    }
    if (lane == 0) {
      s_v[0][wv] = mn; s_v[1][wv] = mx; s_v[2][wv] = smx; s_v[3][wv] = hz;
      s_v[4][wv] = amx; s_v[5][wv] = atot; s_v[6][wv] = ahz;
    }
    __syncthreads();
    if (wv == 0) {  // wave 0: the waves' values, then the zone / domain maxima
      const bool in = lane < ONE_WAVES;
      int64_t a = in ? s_v[0][lane] : 0, b = in ? s_v[1][lane] : 0, d = in ? s_v[2][lane] : 0, e = in ? s_v[3][lane] : 0;
      int64_t f = in ? s_v[4][lane] : 0, g = in ? s_v[5][lane] : 0, q = in ? s_v[6][lane] : 0;
      int64_t zm = 0, am = 0;
      if (ipa.sp >= 0)
        for (int z = lane; z < A.n_zone; z += 64) zm = (int64_t)s_z[z] > zm ? (int64_t)s_z[z] : zm;
      if (ipa.ap >= 0)
        for (int z = lane; z < A.n_adom; z += 64) am = (int64_t)s_az[z] > am ? (int64_t)s_az[z] : am;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const int64_t a2 = __shfl_xor(a, o, 64), b2 = __shfl_xor(b, o, 64), d2 = __shfl_xor(d, o, 64);
        const int64_t e2 = __shfl_xor(e, o, 64), z2 = __shfl_xor(zm, o, 64);
        a = a2 < a ? a2 : a; b = b2 > b ? b2 : b; d = d2 > d ? d2 : d; e = e2 > e ? e2 : e; zm = z2 > zm ? z2 : zm;
        const int64_t f2 = __shfl_xor(f, o, 64), g2 = __shfl_xor(g, o, 64), q2 = __shfl_xor(q, o, 64), m2 = __shfl_xor(am, o, 64);
        f = f2 > f ? f2 : f; g += g2; q = q2 > q ? q2 : q; am = m2 > am ? m2 : am;
      }
      if (lane == 0) {
        s_pa[0] = a; s_pa[1] = b; s_pa[2] = d; s_pa[3] = e; s_pa[4] = zm;
        s_pa[5] = f; s_pa[6] = g; s_pa[7] = q; s_pa[8] = am;
      }
    }
    __syncthreads();
    ipa.mn = s_pa[0]; ipa.mx = s_pa[1]; ipa.smx = s_pa[2]; ipa.hz = s_pa[3] != 0; ipa.szmx = s_pa[4];
    if (ipa.ap >= 0) { ipa.amx = s_pa[5]; ipa.atot = s_pa[6]; ipa.ahz = s_pa[7] != 0; ipa.azmx = s_pa[8]; }
#pragma unroll
    for (int k = 0; k < NPT; ++k) {  // eval_one's additions, same order
      if (!fit[k]) continue;
      if (ipa.on) sc[k] = (int64_t)((uint64_t)sc[k] + (uint64_t)ipa.w * (uint64_t)ksim_interpod_score(raw[k], ipa.mn, ipa.mx));
      if (ipa.sp >= 0) {
        const int64_t v = ksim_spread_score(cnt[k], ipa.smx, ipa.hz, zz[k], zz[k] >= 0 ? (int64_t)s_z[zz[k]] : 0, ipa.szmx);
        sc[k] = (int64_t)((uint64_t)sc[k] + (uint64_t)ipa.sw * (uint64_t)v);
      }
      if (ipa.aon) {  // (count and domain loaded again: no registers held across pass A for them)
        const int64_t i = (int64_t)k * ONE_BLOCK + tid;
        const int32_t d = ksim_dom(A, A.aux_key, i);
        const int64_t v = ipa.ap >= 0 ? A.cnt[A.pair_off[ipa.ap] + i] : 0;
        const int64_t ds = (ipa.ap >= 0 && d >= 0) ? (int64_t)s_az[d] : 0;
        sc[k] = (int64_t)((uint64_t)sc[k] +
                          (uint64_t)ipa.aw * (uint64_t)ksim_aux_score(ipa.akind, v, d, ds, ipa.amx, ipa.atot, ipa.ahz, ipa.azmx));
      }
    }
  }

  if (tid < K) {
    s_tv[tid] = pre_tv;
    s_av[tid] = pre_av;
    s_ad[tid] = pre_ad;
  }
  // ---- per-wave statistics: fit count, per reduce class (max, count at max), reasons ----
  int32_t nfit = 0;
#pragma unroll
  for (int k = 0; k < NPT; ++k) nfit += __popcll(__ballot(fit[k]));
  if (lane == 0) s_fit[wv] = nfit;
  for (int q = 0; q < K; ++q) {  // (uniform)
    int64_t v = INT64_MIN;
#pragma unroll
    for (int k = 0; k < NPT; ++k)
      if (fit[k] && cl[k] == q && sc[k] > v) v = sc[k];
    const int64_t wm = wave_max_i64(v);
    int32_t n = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) n += __popcll(__ballot(fit[k] && cl[k] == q && sc[k] == wm));
    if (lane == 0) {
      s_mx[wv][q] = wm;
      s_cnt[wv][q] = (wm == INT64_MIN) ? 0 : n;
    }
  }
  if (c.collect) {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      if (__ballot(rm[k] != 0)) {
        for (int r = 0; r < KSIM_NREASONS; ++r) {
          const int32_t n = __popcll(__ballot((rm[k] >> r) & 1u));
          if (lane == 0 && n) atomicAdd(&s_hist[r], n);
        }
      }
    }
  }
  __syncthreads();

  // ---- the decision (thread 0): findNodesThatFit count, PrioritizeNodes' reduce step, selectHost ----
  if (tid == 0) {
    D.pod = pod;
    D.K = K;
    D.K2 = k2;
    int32_t F = 0;
    for (int w = 0; w < ONE_WAVES; ++w) F += s_fit[w];
    D.fitTotal = F;
    D.node = -1;
    D.winners = 0;
    if (F == 0) {
      D.mode = 0;
    } else if (F == 1) {  // generic_scheduler.go:153-156: no selectHost, no counter bump
      D.mode = 1;
      D.ix = 0;
    } else {
      D.mode = 2;
      int64_t Mq[KSIM_MAX_RCLASS];
      int32_t Cq[KSIM_MAX_RCLASS];
#pragma unroll
      for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
        int64_t m = INT64_MIN;
        int32_t n = 0;
        if (q < K)
          for (int w = 0; w < ONE_WAVES; ++w) {
            const int32_t cw = s_cnt[w][q];
            const int64_t mw = s_mx[w][q];
            if (cw == 0) continue;
            if (mw > m) { m = mw; n = cw; }
            else if (mw == m) n += cw;
          }
        Mq[q] = m;
        Cq[q] = n;
      }
      // reduce priorities over the filtered set (NormalizeReduce), as ksim_scan_kernel
      int64_t mxT = 0, mxA = 0;
#pragma unroll
      for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
        if (q >= K || Cq[q] == 0) continue;
        if (k1 > 1 || c.w[KSIM_W_TAINT_TOLERATION]) mxT = s_tv[q] > mxT ? s_tv[q] : mxT;
        if (k2 > 1 || c.w[KSIM_W_NODE_AFFINITY]) mxA = s_av[q] > mxA ? s_av[q] : mxA;
      }
      int64_t best = INT64_MIN, tot[KSIM_MAX_RCLASS];
#pragma unroll
      for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
        tot[q] = INT64_MIN;
        if (q >= K || Cq[q] == 0) continue;
        uint64_t t = (uint64_t)Mq[q];
        if (c.w[KSIM_W_TAINT_TOLERATION]) t += (uint64_t)c.w[KSIM_W_TAINT_TOLERATION] * (uint64_t)ksim_norm(s_tv[q], mxT, true);
        if (c.w[KSIM_W_NODE_AFFINITY]) t += (uint64_t)c.w[KSIM_W_NODE_AFFINITY] * (uint64_t)ksim_norm(s_av[q], mxA, false);
        t += (uint64_t)s_ad[q];  // NodePreferAvoidPods
        tot[q] = (int64_t)t;
        best = tot[q] > best ? tot[q] : best;
      }
      uint32_t win = 0;
      int64_t C = 0;
#pragma unroll
      for (int q = 0; q < KSIM_MAX_RCLASS; ++q)
        if (q < K && Cq[q] && tot[q] == best) { win |= 1u << q; C += Cq[q]; }
      D.winners = win;
#pragma unroll
      for (int q = 0; q < KSIM_MAX_RCLASS; ++q) D.M[q] = Mq[q];
      const uint64_t li = pre_ctr;  // generic_scheduler.go:192-195
      D.ix = ((li >> 32) == 0 && C < ((int64_t)1 << 32)) ? (int64_t)((uint32_t)li % (uint32_t)C) : (int64_t)(li % (uint64_t)C);
      pre_ctr = li + 1;
      *c.counter = pre_ctr;
    }
  }
  __syncthreads();

  if (D.mode == 0) {
    if (c.collect && c.out_reasons && tid < KSIM_NREASONS) c.out_reasons[pod * KSIM_NREASONS + tid] = s_hist[tid];
  } else {
    // ---- the ix-th match counted from the largest name rank down ----
    const int mode = D.mode;
    const uint32_t win = D.winners;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const bool mt = fit[k] && (mode == 1 || (((win >> cl[k]) & 1u) && sc[k] == D.M[cl[k]]));
      const uint64_t b = __ballot(mt);
      if (lane == 0) s_bm[k][wv] = b;
    }
    __syncthreads();
    if (wv == 0) {
      // entries e = 0.. (NPT x 16) from the top: (k, w) = (NPT - 1 - e / 16, 15 - e % 16); lane l holds EPL of them
      constexpr int E = NPT * ONE_WAVES, EPL = (E + 63) / 64;
      int32_t n[EPL], tot = 0;
#pragma unroll
      for (int j = 0; j < EPL; ++j) {
        const int e = lane * EPL + j;
        n[j] = e < E ? __popcll(s_bm[NPT - 1 - e / ONE_WAVES][ONE_WAVES - 1 - e % ONE_WAVES]) : 0;
        tot += n[j];
      }
      int32_t incl = tot;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
      }
      const int64_t ix = D.ix;
      const int32_t base = incl - tot;
      const bool hold = tot > 0 && ix >= base && ix < incl;
      if (hold) {
        int64_t r = ix - base;
        for (int j = 0; j < EPL; ++j) {
          if (r < n[j]) {
            const int e = lane * EPL + j;
            const int k = NPT - 1 - e / ONE_WAVES, w = ONE_WAVES - 1 - e % ONE_WAVES;
            uint64_t m = s_bm[k][w];
            for (int64_t q = 0; q < r; ++q) m &= ~(1ull << (63 - __clzll(m)));
            D.node = (int64_t)k * ONE_BLOCK + w * 64 + (63 - __clzll(m));
            break;
          }
          r -= n[j];
        }
      }
      const uint64_t held = __ballot(hold);
      if (lane == 0 && !held) atomicOr(c.err, 2);  // inconsistent counts: must never happen
    }
    __syncthreads();
    if (D.node >= 0 && !c.no_commit) {
      if (wv == 0) {
        const int32_t st = ksim_commit_wave(c, P, D.node, lane);
        if (tid == 0) {
          if (ksim_is_vol_pod(c, P)) ksim_vol_commit_body(*c.vol, P, D.node, 1, c.err);
          if (c.out_fit) c.out_fit[1] |= st;
        }
      } else if (wv == 1 && ksim_is_aff_pod(c, P)) {
        if (lane == 0) ksim_svc_commit(*c.aff, P, D.node);  // reads the counts before this commit's adds
        ksim_aff_commit_body(*c.aff, P, D.node, 1, lane, 64);
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    c.out_node[pod] = (int32_t)D.node;
    if (c.out_fit) {  // fit count, error word and lastNodeIndex into the result block
      c.out_fit[0] = D.fitTotal;
      c.out_fit[KSIM_RES_ERR - KSIM_RES_FIT] = __hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      c.out_fit[KSIM_RES_CTR - KSIM_RES_FIT] = (int32_t)(uint32_t)pre_ctr;
      c.out_fit[KSIM_RES_CTR - KSIM_RES_FIT + 1] = (int32_t)(uint32_t)(pre_ctr >> 32);
    }
  }
}

// ---------------------------------------------------------------------------------------
// The per-pod call on a multi-block cluster (ksim_schedule_one, <= 64 blocks): the same
// evaluation, pass A, decision and commit as ksim_scan_kernel, but with no last block.  Every
// block publishes one tagged record (write-through 8-byte words tag:8 | value:56) and reads
// every other block's: pass A's min / max / max count / haveZones / zone sums
// (interpod_affinity.go:218-236, selector_spreading.go:121-174) in one exchange, the decision
// inputs — fit count, per reduce class (max map score, count at it), the reasons of a block that
// fits nothing — in another, and every block then takes the same decision redundantly
// (generic_scheduler.go:136-198, NormalizeReduce reduce.go:29-64): the block holding the ix-th
// match from the top picks the node from its own candidate masks in LDS and commits it.  One
// cross-block hop per exchange instead of the scan's five serial round trips through the last
// block; the pod travels in the kernel arguments.  All blocks co-resident (host-checked).
namespace {
__device__ __forceinline__ uint64_t pk_enc(uint32_t tag, int64_t v) {
  return ((uint64_t)tag << 56) | ((uint64_t)v & ((1ull << 56) - 1));
}
__device__ __forceinline__ int64_t pk_dec(uint64_t w) { return ((int64_t)(w << 8)) >> 8; }
__device__ __forceinline__ uint32_t pk_tag(uint64_t w) { return (uint32_t)(w >> 56); }
__device__ __forceinline__ void pk_store(uint64_t* g, uint64_t v) {
  __hip_atomic_store(g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t pk_load(const uint64_t* g) {
  return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr uint64_t PK_SPIN_TICKS = 200000000ull;  // 2 s of s_memrealtime
constexpr int PK_BATCH = 16;  // record words one lane keeps in flight (a cross-XCD load is ~1 µs)
// The resident form's answer (ksim_serve_kernel; KsimServeBox::ans in host memory): lane k of the
// answering wave stores result word k (KSIM_RES_*) as `value | seq << 32` in one 8-byte
// system-scope store.  The host takes the answer when every word it reads carries the message's
// number, so no word of an earlier answer can pass for this one whatever order the stores become
// visible in (round 5's answer — untagged words, then a `done` word — needed a system-scope release
// between them).  vr: lane r's FitError reason count (r < KSIM_NREASONS).
// tent: a tentative commit's answer, whose first two reason words carry the row's port count and
// flags before the commit (vr of lanes 0 and 1)
__device__ __forceinline__ void pk_answer(uint64_t* ans, uint64_t seq, int lane, int32_t node, int32_t fit,
                                          int32_t status, int32_t err, uint64_t ctr, int32_t vr, bool tent = false) {
  const int32_t reason = __shfl(vr, (lane - KSIM_RES_REASONS) & 63, 64);
  int32_t v = 0;
  if (lane == KSIM_RES_NODE) v = node;
  else if (lane == KSIM_RES_FIT) v = fit;
  else if (lane == KSIM_RES_STATUS) v = status;
  else if (lane == KSIM_RES_ERR) v = err;
  else if (lane >= KSIM_RES_REASONS && lane < KSIM_RES_REASONS + KSIM_NREASONS) v = reason;
  else if (lane == KSIM_RES_CTR) v = (int32_t)(uint32_t)ctr;
  else if (lane == KSIM_RES_CTR + 1) v = (int32_t)(uint32_t)(ctr >> 32);
  // the reason words only for a FitError (the host reads them only then)
  const bool want = lane < KSIM_RES_WORDS && (node == -1 || lane < KSIM_RES_REASONS || lane >= KSIM_RES_CTR ||
                                               (tent && lane < KSIM_RES_REASONS + 2));
  if (want) __hip_atomic_store(ans + lane, ((uint64_t)(uint32_t)seq << 32) | (uint64_t)(uint32_t)v, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
}
static_assert(KSIM_RES_WORDS <= 64, "one answer word per lane");
}  // namespace

// The thread that caches row `node` (if this block holds it) reloads it after a commit / undo.
template <int NPT>
__device__ __forceinline__ void ksim_row_cache_reload(const KsimCtx& c, KsimRowCache<NPT>& rc, int64_t base, int64_t node) {
  const int64_t j = node - base;
  if (j < 0 || j >= (int64_t)NPT * KSIM_BLOCK || (int)(j % KSIM_BLOCK) != (int)threadIdx.x) return;
  const int kk = (int)(j / KSIM_BLOCK);
#pragma unroll
  for (int k = 0; k < NPT; ++k)
    if (k == kk) rc.r[k] = ksim_load_row(c, node);
}

// One pod of the pick form.  rec: this pod's record buffer (tag parity, KSIM_PICK_WORDS words);
// ctr_keep: the block's own copy of lastNodeIndex (resident form; null: read *c.counter);
// ans / seq: the resident form's answer words and message number (null: a one-pod launch, which
// writes the result block and *c.counter directly); tent: the block's tentative-commit record
// (resident form; no_commit == KSIM_SERVE_TENTATIVE: commit, record, answer the row's prior state).
template <int NPT, bool AUX>
__device__ __forceinline__ void ksim_pick_body(const KsimCtx& c, const ksim_pod& P, const int64_t pod, const uint32_t tag,
                                               const int32_t no_commit, uint64_t* const rec, uint64_t* ctr_keep,
                                               uint64_t* ans, const uint64_t seq, KsimTentRec* tent = nullptr,
                                               KsimRowCache<NPT>* rcache = nullptr, uint64_t* stamp = nullptr) {
#ifdef KSIM_STAMPS
#define PKST(k) do { if (stamp && threadIdx.x == 0) stamp[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define PKST(k) do { (void)stamp; } while (0)
#endif
  __shared__ uint64_t s_bm[KSIM_MAX_RCLASS + 1][NPT][KSIM_WAVES];  // per class (and [MAX] = fit) candidate masks
  __shared__ int64_t s_mx[KSIM_WAVES][KSIM_MAX_RCLASS];
  __shared__ int32_t s_cnt[KSIM_WAVES][KSIM_MAX_RCLASS];
  __shared__ int32_t s_fit[KSIM_WAVES];
  __shared__ int32_t s_hist[KSIM_NREASONS];
  __shared__ int64_t s_v[7][KSIM_WAVES];
  __shared__ unsigned long long s_z[KSIM_PICK_ZMAX];
  __shared__ unsigned long long s_az[KSIM_PICK_ZMAX];  // the auxiliary priority's domain sums
  __shared__ int64_t s_pa[7];
  __shared__ int64_t s_tv[KSIM_MAX_RCLASS], s_av[KSIM_MAX_RCLASS], s_ad[KSIM_MAX_RCLASS];
  __shared__ int64_t s_bmax[KSIM_MAX_RCLASS];  // this block's max per class (after the decision: the winners')
  __shared__ int32_t s_mode, s_owner, s_rank, s_F, s_ok, s_stat;
  __shared__ uint32_t s_win;
  __shared__ int64_t s_M[KSIM_MAX_RCLASS];
  __shared__ int32_t s_C[KSIM_MAX_RCLASS];
  __shared__ int64_t s_rec[KSIM_PICK_MAXG][1 + 2 * KSIM_MAX_RCLASS];  // every block's decision record
  __shared__ uint64_t s_ctr;

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int G = gridDim.x, me = blockIdx.x;
  const int k1 = P.reserved[0], k2 = P.reserved[1];
  const int K = k1 * k2;  // <= KSIM_MAX_RCLASS (host-checked)
  uint64_t* const recA = rec;
  uint64_t* const recB = rec + KSIM_PICK_MAXG * KSIM_PICK_RA;
  // the decision's inputs, loaded while the nodes are evaluated
  int64_t pre_tv = 0, pre_av = 0, pre_ad = 0;
  if (tid < K) {
    pre_tv = c.tt_val[(int64_t)P.cls * c.val_w + tid / k2];
    pre_av = c.na_val[(int64_t)P.cls * c.val_w + tid % k2];
    pre_ad = c.na_add ? c.na_add[(int64_t)P.cls * c.val_w + tid % k2] : 0;
  }
  uint64_t pre_ctr = 0;
  if (tid == 0) pre_ctr = ctr_keep ? *ctr_keep : *c.counter;
  IpaNorm ipa = ipa_norm(c, P);  // which of pass A's priorities the pod reads (maxima below)
  IpaNorm ipa0 = ipa;
  ipa0.on = false;
  ipa0.sp = -1;
  ipa0.aon = false;
  // AUX (a compile-time instantiation: the handle has the auxiliary priority's tables): the pod
  // may read the auxiliary priority (the kernels without it keep their registers for the rest)
  const bool pass_a = ipa.on || ipa.sp >= 0 || (AUX && ipa.aon);
  // pass-A record words: 4 maxima, NZ zone sums, then (a pod with an auxiliary count) 3 words and
  // NA domain sums; 4 + NZ + 3 + NA <= KSIM_PICK_RA (host-checked)
  const int NZ = (ipa.sp >= 0) ? c.aff->n_zone : 0;
  const bool AX = AUX && ipa.ap >= 0;
  const int NA = AX ? c.aff->n_adom : 0;
  const int A0 = 4 + NZ;  // the auxiliary words
  __shared__ uint32_t s_dflag;  // the decision is in LDS (wave 0 → the other waves)
  if (tid < KSIM_NREASONS) s_hist[tid] = 0;
  if (tid < KSIM_PICK_ZMAX) {
    s_z[tid] = 0;
    if (AUX) s_az[tid] = 0;
  }
  if (tid == 0) { s_ok = 1; s_dflag = 0; s_stat = 0; }
  __syncthreads();

  const int64_t base = (int64_t)me * c.chunk;
  bool fit[NPT];
  int64_t sc[NPT];
  int cl[NPT];
  uint32_t rm[NPT];
  if (rcache) {  // (uniform) the resident kernel: rows from registers
#pragma unroll
    for (int k = 0; k < NPT; ++k)
      eval_cached<true>(c, P, base + (int64_t)k * KSIM_BLOCK + tid, rcache->r[k], rcache->ls[k], rcache->ts[k], k1, k2, fit[k],
                        sc[k], cl[k], rm[k]);
  } else {
#pragma unroll
    for (int k = 0; k < NPT; ++k) eval_one<true>(c, P, base + (int64_t)k * KSIM_BLOCK + tid, k1, k2, ipa0, fit[k], sc[k], cl[k], rm[k]);
  }

  PKST(2);
  // the first spin that hits its bound: err bit 2 (a consistency error; the grid is co-resident)
  // the first consistency failure of a handle, for the host's error message: dbg[96] =
  // site | me << 8 | tag << 16 | seq << 24, dbg[97] = a detail (KSIM_PICK_NOTE)
  auto note = [&](uint64_t site, uint64_t detail) {
    if (c.dbg && atomicCAS((unsigned long long*)&c.dbg[96], 0ull,
                           (unsigned long long)(site | (uint64_t)me << 8 | (uint64_t)tag << 16 | (seq & 0xffffffffull) << 24)) == 0ull)
      atomicExch((unsigned long long*)&c.dbg[97], (unsigned long long)detail);
  };
  auto spin_fail = [&](int site) {
    if (lane == 0) { atomicOr(c.err, 2); s_ok = 0; note(site, 0); }
  };

  if (pass_a) {  // (uniform) pass A over the fit nodes: the block's partial, then every block's
    const KsimAff& A = *c.aff;
    int64_t raw[NPT], cnt[NPT];
    int32_t zz[NPT];
    int64_t mn = 0, mx = 0, smx = 0, hz = 0, amx = 0, atot = 0, ahz = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int64_t i = base + (int64_t)k * KSIM_BLOCK + tid;
      raw[k] = 0; cnt[k] = 0; zz[k] = -1;
      if (!fit[k]) continue;
      if (ipa.on) {
        raw[k] = ksim_interpod_raw_body(A, P, i);
        mn = raw[k] < mn ? raw[k] : mn;
        mx = raw[k] > mx ? raw[k] : mx;
      }
      if (ipa.sp >= 0) {
        cnt[k] = A.cnt[A.pair_off[ipa.sp] + i];
        zz[k] = A.zone_key >= 0 ? ksim_dom(A, A.zone_key, i) : -1;
        smx = cnt[k] > smx ? cnt[k] : smx;
        if (zz[k] >= 0) {
          hz = 1;
          if (cnt[k]) atomicAdd(&s_z[zz[k]], (unsigned long long)cnt[k]);
        }
      }
      if (AX) {  // the auxiliary priority (passa_reduce's): max, sum, haveZones, domain sums
        const int64_t v = A.cnt[A.pair_off[ipa.ap] + i];
        const int32_t d = ksim_dom(A, A.aux_key, i);
        amx = v > amx ? v : amx;
        atot += v;
        if (d >= 0) {
          ahz = 1;
          if (v) atomicAdd(&s_az[d], (unsigned long long)v);
        }
      }
    }
    mn = ksimw::min_i64(mn);
    mx = ksimw::max_i64(mx);
    smx = ksimw::max_i64(smx);
    hz = ksimw::max_i64(hz);
    if (AX) {  // (uniform)
      amx = ksimw::max_i64(amx);
      atot = ksimw::sum_i64(atot);
      ahz = ksimw::max_i64(ahz);
    }
    if (lane == 0) {
      s_v[0][wv] = mn; s_v[1][wv] = mx; s_v[2][wv] = smx; s_v[3][wv] = hz;
      if (AUX) { s_v[4][wv] = amx; s_v[5][wv] = atot; s_v[6][wv] = ahz; }
    }
    __syncthreads();
    const int W = A0 + (AX ? 3 + NA : 0);
    // word x's combine over waves and blocks: 0 = min, 1 = max, 2 = sum
    const int op = lane == 0 ? 0 : (lane < 4 ? 1 : ((!AUX || lane < A0) ? 2 : (lane == A0 || lane == A0 + 2 ? 1 : 2)));
    if (wv == 1) {
      // publish: word x = lane x (0..3 the maxima over this block's waves, 4.. the zone sums, then
      // the auxiliary max / sum / haveZones and domain sums).  Wave 1 stores, wave 0 polls: a store
      // counts in the storing wave's vmcnt until it is acknowledged, and the poll's loads would
      // otherwise wait for that acknowledgement too.
      int64_t v = 0;
      if (lane < 4 || (AX && lane >= A0 && lane < A0 + 3)) {
        const int row = lane < 4 ? lane : 4 + lane - A0;
        v = s_v[row][0];
        for (int w = 1; w < KSIM_WAVES; ++w) {
          const int64_t x = s_v[row][w];
          v = op == 0 ? (x < v ? x : v) : (op == 1 ? (x > v ? x : v) : v + x);
        }
      } else if (lane < A0) {
        v = (int64_t)s_z[lane - 4];
      } else if (AX && lane < W) {
        v = (int64_t)s_az[lane - A0 - 3];
      }
      // every word of the record, not only the W read now: see the record stores below
      pk_store(recA + (int64_t)me * KSIM_PICK_RA + lane, pk_enc(tag, lane < W ? v : 0));
    }
    if (wv == 0) {
      // every block's record: lane x combines word x over the blocks
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      int64_t acc = 0;
      for (;;) {
        bool ok = true;
        acc = 0;  // (0 folded into every combine: the reference's accumulators start there)
        for (int b0 = 0; b0 < G && lane < W; b0 += PK_BATCH) {
          uint64_t wd[PK_BATCH];  // one batch of blocks' words in flight: one round trip per batch
#pragma unroll
          for (int j = 0; j < PK_BATCH; ++j)
            wd[j] = b0 + j < G ? pk_load(recA + (int64_t)(b0 + j) * KSIM_PICK_RA + lane) : pk_enc(tag, 0);
#pragma unroll
          for (int j = 0; j < PK_BATCH; ++j) {
            if (b0 + j >= G) break;
            ok &= pk_tag(wd[j]) == tag;
            const int64_t x = pk_dec(wd[j]);
            acc = op == 0 ? (x < acc ? x : acc) : (op == 1 ? (x > acc ? x : acc) : acc + x);
          }
        }
        if (__all(ok)) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > PK_SPIN_TICKS) { spin_fail(1); break; }
        __builtin_amdgcn_s_sleep(1);
      }
      if (lane < 4) s_pa[lane] = acc;
      else if (lane < A0) s_z[lane - 4] = (unsigned long long)acc;
      else if (lane < A0 + 3 && AX) s_pa[4 + lane - A0] = acc;
      else if (AX && lane < W) s_az[lane - A0 - 3] = (unsigned long long)acc;
    }
    __syncthreads();
    ipa.mn = s_pa[0]; ipa.mx = s_pa[1]; ipa.smx = s_pa[2]; ipa.hz = s_pa[3] != 0;
    int64_t zm = 0;  // the zone maximum (over every zone: zeros included, as the scan's pass A)
    for (int z = 0; z < NZ; ++z) zm = (int64_t)s_z[z] > zm ? (int64_t)s_z[z] : zm;
    ipa.szmx = zm;
    if (AX) {  // (the auxiliary domain maximum likewise)
      int64_t am = 0;
      for (int z = 0; z < NA; ++z) am = (int64_t)s_az[z] > am ? (int64_t)s_az[z] : am;
      ipa.amx = s_pa[4]; ipa.atot = s_pa[5]; ipa.ahz = s_pa[6] != 0; ipa.azmx = am;
    }
#pragma unroll
    for (int k = 0; k < NPT; ++k) {  // eval_one's additions, same order
      if (!fit[k]) continue;
      if (ipa.on) sc[k] = (int64_t)((uint64_t)sc[k] + (uint64_t)ipa.w * (uint64_t)ksim_interpod_score(raw[k], ipa.mn, ipa.mx));
      if (ipa.sp >= 0) {
        const int64_t v = ksim_spread_score(cnt[k], ipa.smx, ipa.hz, zz[k], zz[k] >= 0 ? (int64_t)s_z[zz[k]] : 0, ipa.szmx);
        sc[k] = (int64_t)((uint64_t)sc[k] + (uint64_t)ipa.sw * (uint64_t)v);
      }
      if (AUX && ipa.aon) {  // (count and domain loaded again: no registers held across pass A for them)
        const int64_t i = base + (int64_t)k * KSIM_BLOCK + tid;
        const int32_t d = ksim_dom(A, A.aux_key, i);
        const int64_t v = AX ? A.cnt[A.pair_off[ipa.ap] + i] : 0;
        const int64_t ds = (AX && d >= 0) ? (int64_t)s_az[d] : 0;
        sc[k] = (int64_t)((uint64_t)sc[k] +
                          (uint64_t)ipa.aw * (uint64_t)ksim_aux_score(ipa.akind, v, d, ds, ipa.amx, ipa.atot, ipa.ahz, ipa.azmx));
      }
    }
  }

  PKST(3);
  if (tid < K) { s_tv[tid] = pre_tv; s_av[tid] = pre_av; s_ad[tid] = pre_ad; }
  if (tid == 0) s_ctr = pre_ctr;
  // ---- per wave: fit count and mask, per reduce class (max, count at max) and masks, reasons ----
  int32_t nfit = 0;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const uint64_t b = __ballot(fit[k]);
    nfit += __popcll(b);
    if (lane == 0) s_bm[KSIM_MAX_RCLASS][k][wv] = b;
  }
  if (lane == 0) s_fit[wv] = nfit;
  for (int q = 0; q < K; ++q) {  // (uniform)
    int64_t v = INT64_MIN;
#pragma unroll
    for (int k = 0; k < NPT; ++k)
      if (fit[k] && cl[k] == q && sc[k] > v) v = sc[k];
    const int64_t wm = ksimw::max_i64(v);
    int32_t n = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const uint64_t b = __ballot(fit[k] && cl[k] == q && sc[k] == wm);
      n += __popcll(b);
      if (lane == 0) s_bm[q][k][wv] = b;
    }
    if (lane == 0) { s_mx[wv][q] = wm; s_cnt[wv][q] = wm == INT64_MIN ? 0 : n; }
  }
  __syncthreads();
  // the reasons histogram only when this block fits nothing (it is published only then)
  const int32_t F0 = s_fit[0] + s_fit[1] + s_fit[2] + s_fit[3];
  if (F0 == 0) {  // (uniform)
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      if (__ballot(rm[k] != 0)) {
        for (int r = 0; r < KSIM_NREASONS; ++r) {
          const int32_t n = __popcll(__ballot((rm[k] >> r) & 1u));
          if (lane == 0 && n) atomicAdd(&s_hist[r], n);
        }
      }
    }
    __syncthreads();
  }

  if (wv <= 1) {
    // ---- this block's record: fit, per class (max, count), reasons when it fits nothing; wave 1
    // stores it, wave 0 keeps the per-class maxima and polls (see pass A) ----
    int64_t bm = INT64_MIN;
    int32_t bc = 0;
    if (lane < K) {
      for (int w = 0; w < KSIM_WAVES; ++w) {
        if (s_cnt[w][lane] == 0) continue;
        if (s_mx[w][lane] > bm) { bm = s_mx[w][lane]; bc = s_cnt[w][lane]; }
        else if (s_mx[w][lane] == bm) bc += s_cnt[w][lane];
      }
      if (wv == 0) s_bmax[lane] = bc ? bm : INT64_MIN;
    }
    if (wv == 1) {
      // Every word of both records carries this call's tag after this call, including words no
      // block reads now (zeros): the tags (1..254) come back every 254 calls, so a word written
      // by an older call and not since would pass for this call's if a later pod read further
      // into the record (more reduce classes K, more zones, a pod with pass A after pods without).
      const int WB = 1 + 2 * K + (F0 == 0 ? KSIM_NREASONS : 0);
      // word x = lane x: fit, then class q's max (word 1 + q), its count (word 1 + K + q), reasons
      const int64_t mq = __shfl(bm, (lane - 1) & 63, 64);
      const int32_t cq = __shfl(bc, (lane - 1) & 63, 64), cq2 = __shfl(bc, (lane - 1 - K) & 63, 64);
      int64_t v = 0;
      if (lane == 0) v = F0;
      else if (lane <= K) v = cq ? mq : 0;  // (a class without fit nodes: count 0, max unread)
      else if (lane <= 2 * K) v = cq2;
      else if (lane < WB) v = s_hist[lane - 1 - 2 * K];
      if (!pass_a) pk_store(recA + (int64_t)me * KSIM_PICK_RA + lane, pk_enc(tag, 0));
      pk_store(recB + (int64_t)me * KSIM_PICK_RB + lane, pk_enc(tag, v));
      // word 64 (the last reason when K = 16) from lane 0
      static_assert(KSIM_PICK_RB == 65 && KSIM_PICK_RA == 64, "record words per lane");
      if (lane == 0) pk_store(recB + (int64_t)me * KSIM_PICK_RB + 64, pk_enc(tag, 64 < WB ? s_hist[64 - 1 - 2 * K] : 0));
    }
  }
  if (wv == 0) {
    PKST(4);
    // ---- every block's record (lane b = block b, staged in LDS), then the decision, the same in
    // every block ----
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      bool ok = true;
      if (lane < G)
        for (int x0 = 0; x0 <= 2 * K; x0 += PK_BATCH) {
          uint64_t w[PK_BATCH];  // one batch of words in flight: one round trip per batch
#pragma unroll
          for (int j = 0; j < PK_BATCH; ++j)
            w[j] = x0 + j <= 2 * K ? pk_load(recB + (int64_t)lane * KSIM_PICK_RB + x0 + j) : pk_enc(tag, 0);
#pragma unroll
          for (int j = 0; j < PK_BATCH; ++j) {
            if (x0 + j > 2 * K) break;
            ok &= pk_tag(w[j]) == tag;
            s_rec[lane][x0 + j] = pk_dec(w[j]);
          }
        }
      if (__all(ok)) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > PK_SPIN_TICKS) { spin_fail(2); break; }
      __builtin_amdgcn_s_sleep(1);
    }
    PKST(5);
    const bool in = lane < G;
    const int32_t fb = in ? (int32_t)s_rec[lane][0] : 0;
    const int32_t F = ksimw::sum_i32(fb);
    int mode = F == 0 ? 0 : (F == 1 ? 1 : 2);
    uint32_t win = 0;
    int64_t C = 0;
    if (mode == 2) {
      for (int q = 0; q < K; ++q) {  // (uniform) the grid's max and count per class
        const int32_t cb = in ? (int32_t)s_rec[lane][1 + K + q] : 0;
        const int64_t mb = cb ? s_rec[lane][1 + q] : INT64_MIN;
        const int64_t m = ksimw::max_i64(mb);
        const int32_t n = ksimw::sum_i32((cb && mb == m) ? cb : 0);
        if (lane == 0) { s_M[q] = m; s_C[q] = n; }
      }
      PKST(6);
      // reduce priorities over the filtered set (NormalizeReduce), as ksim_scan_kernel, lane q =
      // class q: the maxima over the live classes and the winners by wave reductions
      const bool live = lane < K && s_C[lane] > 0;
      const int64_t tvq = lane < K ? s_tv[lane] : 0, avq = lane < K ? s_av[lane] : 0;
      const int64_t mxT = ksimw::max_i64(live && (k1 > 1 || c.w[KSIM_W_TAINT_TOLERATION]) ? tvq : 0);
      const int64_t mxA = ksimw::max_i64(live && (k2 > 1 || c.w[KSIM_W_NODE_AFFINITY]) ? avq : 0);
      int64_t tot = INT64_MIN;
      if (live) {
        uint64_t t = (uint64_t)s_M[lane];
        if (c.w[KSIM_W_TAINT_TOLERATION]) t += (uint64_t)c.w[KSIM_W_TAINT_TOLERATION] * (uint64_t)ksim_norm(tvq, mxT, true);
        if (c.w[KSIM_W_NODE_AFFINITY]) t += (uint64_t)c.w[KSIM_W_NODE_AFFINITY] * (uint64_t)ksim_norm(avq, mxA, false);
        t += (uint64_t)s_ad[lane];  // NodePreferAvoidPods
        tot = (int64_t)t;
      }
      const int64_t best = ksimw::max_i64(tot);
      const bool w_q = live && tot == best;
      win = (uint32_t)__ballot(w_q);
      C = ksimw::sum_i32(w_q ? s_C[lane] : 0);
    }
    // selectHost: the ix-th match counted from the largest name rank down (blocks from the top)
    const uint64_t li = s_ctr;
    int64_t ix = 0;
    if (mode == 2) ix = ((li >> 32) == 0 && C < ((int64_t)1 << 32)) ? (int64_t)((uint32_t)li % (uint32_t)C) : (int64_t)(li % (uint64_t)C);
    int64_t mt = 0;  // this lane's block: its matches
    if (in && mode == 1) mt = fb;
    if (in && mode == 2)
      for (int q = 0; q < K; ++q) {
        if (!((win >> q) & 1u)) continue;
        const int32_t cb = (int32_t)s_rec[lane][1 + K + q];
        if (cb && s_rec[lane][1 + q] == s_M[q]) mt += cb;
      }
    const int32_t incl = ksimw::prefix_incl_i32((int32_t)mt);
    const int32_t total = __builtin_amdgcn_readlane(incl, 63);
    // blocks from the top: block b's matches come after those of every block above it
    const int32_t above = total - incl;
    const uint64_t hb = __ballot(mode != 0 && mt > 0 && ix >= above && ix < above + mt);
    const int owner = hb ? 63 - __builtin_clzll(hb) : -1;
    const int32_t rank = owner >= 0 ? (int32_t)ix - __builtin_amdgcn_readlane(above, owner) : 0;
    if (lane == 0) {
      if (mode != 0 && owner < 0) {  // inconsistent counts: must never happen
        atomicOr(c.err, 2);
        note(4, (uint64_t)(uint32_t)total << 32 | (uint64_t)(uint32_t)C);
        mode = 0;
      }
      s_mode = s_ok ? mode : -1;
      s_owner = owner;
      s_rank = rank;
      s_F = F;
      s_win = win;
      s_ctr = (mode == 2) ? li + 1 : li;  // generic_scheduler.go:192-195
      if (ctr_keep) *ctr_keep = s_ctr;
    }
    if (mode != 2 && lane < KSIM_MAX_RCLASS) s_M[lane] = INT64_MIN;
    // the decision to the other waves through an LDS flag, not a barrier: a barrier would also
    // wait for wave 1's record store to be acknowledged (the waits before s_barrier)
    if (lane == 0) __hip_atomic_store(&s_dflag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
    while (__hip_atomic_load(&s_dflag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) __builtin_amdgcn_s_sleep(1);
  }
  PKST(7);
  const int mode = s_mode;
  if (mode < 0) {  // a spin hit its bound (err set): nothing committed
    if (ans && me == 0 && wv == 0)  // (the resident form: the host must hear of it)
      pk_answer(ans, seq, lane, INT32_MIN, 0, 0, __hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) | 2, s_ctr, 0);
    return;
  }

  if (mode == 0) {
    if (me == 0 && wv == 0) {  // FitError: every block's reasons (each fitted nothing)
      int32_t v = 0;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {  // (the reason words went out in the same store as the words read above, tagged alike)
        bool ok = true;
        v = 0;
        for (int b0 = 0; b0 < G && lane < KSIM_NREASONS; b0 += PK_BATCH) {
          uint64_t wd[PK_BATCH];  // one batch of blocks' words in flight
#pragma unroll
          for (int j = 0; j < PK_BATCH; ++j)
            wd[j] = b0 + j < G ? pk_load(recB + (int64_t)(b0 + j) * KSIM_PICK_RB + 1 + 2 * K + lane) : pk_enc(tag, 0);
#pragma unroll
          for (int j = 0; j < PK_BATCH; ++j) {
            if (b0 + j >= G) break;
            ok &= pk_tag(wd[j]) == tag;
            v += (int32_t)pk_dec(wd[j]);
          }
        }
        if (__all(ok)) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > PK_SPIN_TICKS) { atomicOr(c.err, 2); if (lane == 0) note(3, 0); break; }
        __builtin_amdgcn_s_sleep(1);
      }
      const int32_t e = __hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ans) {
        pk_answer(ans, seq, lane, -1, 0, 0, e, s_ctr, v);
      } else {
        if (lane < KSIM_NREASONS) c.out_reasons[pod * KSIM_NREASONS + lane] = v;
        if (lane == 0) {
          c.out_node[pod] = -1;
          if (c.out_fit) {
            c.out_fit[0] = 0;
            c.out_fit[KSIM_RES_ERR - KSIM_RES_FIT] = e;
            c.out_fit[KSIM_RES_CTR - KSIM_RES_FIT] = (int32_t)(uint32_t)s_ctr;
            c.out_fit[KSIM_RES_CTR - KSIM_RES_FIT + 1] = (int32_t)(uint32_t)(s_ctr >> 32);
          }
        }
      }
      PKST(10);
    }
    return;
  }
  if (me != s_owner) return;

  // ---- the owner block: its rank-th match from the top, from its own candidate masks ----
  __shared__ int64_t s_node;
  if (wv == 0) {
    // lane t = (k, w) segment from the top: its mask of matches
    uint64_t m = 0;
    const int k = NPT - 1 - lane / KSIM_WAVES, w = KSIM_WAVES - 1 - lane % KSIM_WAVES;
    if (lane < NPT * KSIM_WAVES) {
      if (mode == 1) {
        m = s_bm[KSIM_MAX_RCLASS][k][w];
      } else {
        for (int q = 0; q < K; ++q)
          if (((s_win >> q) & 1u) && s_bmax[q] == s_M[q] && s_mx[w][q] == s_M[q]) m |= s_bm[q][k][w];
      }
    }
    const int32_t n = __popcll(m);
    const int32_t incl = ksimw::prefix_incl_i32(n);
    const int32_t r = s_rank;
    const bool here = n > 0 && r >= incl - n && r < incl;
    const uint64_t hs = __ballot(here);
    int64_t node = -1;
    if (hs) {
      const int t = __builtin_ctzll(hs);
      const uint64_t ms = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(m >> 32), t) << 32) |
                          (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)m, t);
      const int32_t rr = r - (__builtin_amdgcn_readlane(incl, t) - __popcll(ms));
      const uint64_t hb2 = __ballot(((ms >> lane) & 1ull) && __popcll(ms >> lane) - 1 == rr);
      const int kt = NPT - 1 - t / KSIM_WAVES, wt = KSIM_WAVES - 1 - t % KSIM_WAVES;
      if (hb2) node = (int64_t)me * c.chunk + (int64_t)kt * KSIM_BLOCK + wt * 64 + __builtin_ctzll(hb2);
    }
    if (lane == 0) {
      if (node < 0) { atomicOr(c.err, 2); note(5, (uint64_t)(uint32_t)s_rank); }  // inconsistent masks: must never happen
      s_node = node;
    }
  }
  __syncthreads();
  PKST(8);
  const int64_t node = s_node;
  const bool tentative = tent && no_commit == KSIM_SERVE_TENTATIVE;
  __shared__ int32_t s_cnt0;
  __shared__ uint32_t s_fl0;
  if (node >= 0 && no_commit != 1) {
    // a commit of state other blocks read (volume mounts, inter-pod affinity / service counts): each
    // committing wave releases it at agent scope before the answer, so the next message's acquire
    // (KSIM_SERVE_SYNC_ACQUIRE) sees it (rows are read by this block's own waves only)
    if (wv == 0) {
      int32_t cnt0 = 0;
      uint32_t fl0 = 0;
      if (tentative && lane == 0) { cnt0 = c.port_count[node]; fl0 = c.flags[node]; }
      const int32_t st = ksim_commit_wave(c, P, node, lane);
      if (tid == 0) {
        if (ksim_is_vol_pod(c, P)) ksim_vol_commit_body(*c.vol, P, node, 1, c.err);
        s_stat = st;
        if (tentative) {
          s_cnt0 = cnt0;
          s_fl0 = fl0;
          tent->node = node;
          tent->seq = (uint32_t)seq;
          tent->cnt0 = cnt0;
          tent->fl0 = fl0;
          tent->P = P;
          for (int32_t k = 0; k < P.scalar_cnt; ++k) tent->sc[k] = ksim_pod_scalar(c, P, k);
          tent->valid = 1;
        }
      }
      if (ans && ksim_is_vol_pod(c, P)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    } else if (wv == 1 && ksim_is_aff_pod(c, P)) {
      if (lane == 0) ksim_svc_commit(*c.aff, P, node);  // reads the counts before this commit's adds
      ksim_aff_commit_body(*c.aff, P, node, 1, lane, 64);
      if (ans) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    }
  }
  __syncthreads();
  PKST(9);
  if (ans) {
    // the answer; lastNodeIndex stays in the blocks' LDS (every block took the same decision) and
    // reaches the host in the answer — no device store of it while the kernel is resident
    if (wv == 0) {
      const bool tc = tentative && node >= 0;
      pk_answer(ans, seq, lane, (int32_t)node, s_F, s_stat, __hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                s_ctr, tc ? (lane == 0 ? s_cnt0 : (int32_t)s_fl0) : 0, tc);
    }
    // the committed row's register copy (after the answer: off the decision chain; the commit's
    // stores are this workgroup's own, ordered by the barrier above)
    if (rcache && node >= 0 && no_commit != 1) ksim_row_cache_reload<NPT>(c, *rcache, base, node);
  } else if (tid == 0) {
    if (mode == 2) *c.counter = s_ctr;  // (a one-pod launch: this block is the call's only writer)
    c.out_node[pod] = (int32_t)node;
    if (c.out_fit) {
      if (s_stat) c.out_fit[1] |= s_stat;
      c.out_fit[0] = s_F;
      c.out_fit[KSIM_RES_ERR - KSIM_RES_FIT] = __hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      c.out_fit[KSIM_RES_CTR - KSIM_RES_FIT] = (int32_t)(uint32_t)s_ctr;
      c.out_fit[KSIM_RES_CTR - KSIM_RES_FIT + 1] = (int32_t)(uint32_t)(s_ctr >> 32);
    }
  }
  if (tid == 0) PKST(10);
#undef PKST
}

template <int NPT, bool AUX>
__global__ __launch_bounds__(KSIM_BLOCK) void ksim_pick_kernel(KsimCtx c) {
  ksim_pick_body<NPT, AUX>(c, c.one_pod, c.first, c.pick_tag, c.no_commit, c.pick + (c.pick_tag & 1u) * KSIM_PICK_WORDS,
                      nullptr, nullptr, 0);
}

// ---------------------------------------------------------------------------------------
// The resident per-pod service (ksim_schedule_one / ksim_pod_add between other calls): the pick
// kernel's grid stays resident and takes one message at a time from a mailbox in coherent host
// memory (KsimServeBox: tagged words, one PCIe round trip per poll), so a call costs the host's
// stores, the device's poll and the answer's stores instead of a kernel launch and a stream
// synchronisation.  Each block copies the message's pod into its own slot of the device staging
// (c.pods / c.pod_ports / c.pod_scalars, one slot per block: the evaluation reads its ports /
// scalars there), keeps lastNodeIndex in LDS (every block takes every SCHEDULE message and the
// same decision), and uses the record buffer of the message's tag parity, so a block still
// reading pod k's records never sees them overwritten by pod k + 1's.  The grid leaves on an exit
// message or by the idle vote (KSIM_SERVE_ST_*, ksim_common.h).
namespace {
// The idle vote, lane 0 of a block's wave 0 (agent-scope atomics on one device word).
// serve_vote: this block's vote; 2 = it made the vote unanimous (LEFT set), 1 = counted in epoch
// *ep, 0 = the grid had already left (cannot happen: LEFT needs this block's vote).
__device__ uint32_t serve_vote(uint64_t* st, uint32_t G, uint32_t* ep) {
  uint64_t s = __hip_atomic_load(st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    if (s & KSIM_SERVE_ST_LEFT) return 0;
    const uint32_t v = KSIM_SERVE_ST_VOTES(s) + 1;
    const uint64_t n = v >= G ? (s | KSIM_SERVE_ST_LEFT) : KSIM_SERVE_ST_MAKE(KSIM_SERVE_ST_EPOCH(s), v);
    if (__hip_atomic_compare_exchange_strong(st, &s, n, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
      *ep = KSIM_SERVE_ST_EPOCH(s);
      return v >= G ? 2u : 1u;
    }
  }
}
// serve_veto: withdraw this block's vote of epoch ep before taking a message (bump the epoch,
// clear the votes); 1 = take it, 0 = the grid agreed to leave before (the message is not taken).
__device__ uint32_t serve_veto(uint64_t* st, uint32_t ep) {
  uint64_t s = __hip_atomic_load(st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    if (s & KSIM_SERVE_ST_LEFT) return 0;
    if (KSIM_SERVE_ST_EPOCH(s) != ep) return 1;  // another block's veto already cleared the votes
    if (__hip_atomic_compare_exchange_strong(st, &s, KSIM_SERVE_ST_MAKE(ep + 1u, 0u), __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      return 1;
  }
}
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(v >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)v);
}
}  // namespace

template <int NPT, bool AUX>
__global__ __launch_bounds__(KSIM_BLOCK) void ksim_serve_kernel(KsimCtx c, KsimServeArgs a) {
  __shared__ uint64_t s_keep;
  __shared__ ksim_pod s_P;
  __shared__ int32_t s_type, s_nc;
  __shared__ uint32_t s_tag;
  __shared__ int64_t s_node;
  __shared__ uint32_t s_msg[KSIM_SERVE_MSG_WORDS];
  __shared__ uint64_t s_seq;
  __shared__ KsimTentRec s_tent;  // this block's tentative commit awaiting the host's decision
  __shared__ int32_t s_got;       // wave 0 took a message (an EXIT included)
  __shared__ int32_t s_undid;     // this message undid this block's tentative commit
  KsimServeBox* const box = a.box;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, me = blockIdx.x;
  // lastNodeIndex: from the host's last answer, or (after calls of other forms) the device word,
  // read coherently (system scope: never a stale line of this XCD's L2)
  if (tid == 0) {
    s_keep = a.ctr0_valid ? a.ctr0 : __hip_atomic_load(c.counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    s_tent.valid = 0;
  }
#ifdef KSIM_STAMPS
  // diagnostic builds: per phase, the sum of (stamp k - stamp k-1) and how often both were taken,
  // over every block and message, into dbg[64 + k] / dbg[80 + k] at the exit (k = 0: the poll)
  __shared__ uint64_t s_st[12], s_sum[12], s_cnt[12];
  uint64_t* const stamp = s_st;
  if (tid < 12) { s_sum[tid] = 0; s_cnt[tid] = 0; s_st[tid] = 0; }
  uint64_t n_polls = 0;
  uint64_t t_end = __builtin_amdgcn_s_memrealtime();
#else
  uint64_t* const stamp = nullptr;
#endif
  uint64_t* const pod_ports = const_cast<uint64_t*>(c.pod_ports) + (int64_t)me * KSIM_ONE_PORTS;
  ksim_scalar_req* const pod_scalars = const_cast<ksim_scalar_req*>(c.pod_scalars) + (int64_t)me * KSIM_MAX_SCALAR;
  // this thread's rows for the kernel's lifetime (KsimRowCache)
  const int64_t base = (int64_t)me * c.chunk;
  KsimRowCache<NPT> rcache;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int64_t i = base + (int64_t)k * KSIM_BLOCK + tid;
    if (i < c.n) {
      rcache.r[k] = ksim_load_row(c, i);
      rcache.ls[k] = c.label_set[i];
      rcache.ts[k] = c.taint_set[i];
    } else {
      rcache.r[k] = KsimRow{};
      rcache.ls[k] = rcache.ts[k] = 0;
    }
  }
  // A block takes the newest complete message, which may be past the next one: a message answered
  // by one block (an assume onto another block's node) does not wait for the others, so the host
  // can post the next before this block has looked.  It never skips one it must answer or publish
  // records for: the host waits for those.
  uint64_t seq = a.seq0;
  bool voted = false;  // (wave 0, uniform) this block's idle vote stands in epoch vote_ep
  uint32_t vote_ep = 0;
  uint64_t t_idle = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (wv == 0) {
      // poll: lane l reads payload words 2l, 2l+1 with their tags in one 16-byte system-scope load
      typedef unsigned int u4 __attribute__((ext_vector_type(4)));
      const uint32_t s32 = (uint32_t)seq + 1u;  // the oldest message this block may take
      const uint64_t* src = box->msg + 2 * lane;
      u4 q;
      int32_t type = KSIM_SERVE_EXIT;
      bool got = false;
      for (;;) {
        asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(q) : "v"(src) : "memory");
        const uint32_t t = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)q.y);
        if ((int32_t)(t - s32) >= 0 && __all(q.y == t && q.w == t)) {
          type = __builtin_amdgcn_readfirstlane((int32_t)q.x);  // word 0 (lane 0)
          got = true;
          if (type != KSIM_SERVE_EXIT && voted) {
            // this block voted to leave: withdraw the vote before taking the message
            uint32_t ok = 0;
            if (lane == 0) ok = serve_veto(a.state, vote_ep);
            ok = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)ok);
            voted = false;
            if (!ok) { type = KSIM_SERVE_EXIT; got = false; }  // the grid left first: nobody takes it (the host relaunches)
          }
          if (lane == 0) s_seq = seq + 1 + (uint64_t)(t - s32);
#ifdef KSIM_STAMPS
          if (lane == 0) s_st[0] = __builtin_amdgcn_s_memrealtime();
#endif
          break;
        }
        const uint64_t now = __builtin_amdgcn_s_memrealtime();  // (uniform: one clock read per wave)
        if (voted) {
          // the vote stands until every block voted (LEFT) or a block saw a message (new epoch)
          uint64_t sv = 0;
          if (lane == 0) sv = __hip_atomic_load(a.state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          sv = rfl64(sv);
          if (sv & KSIM_SERVE_ST_LEFT) break;
          if (KSIM_SERVE_ST_EPOCH(sv) != vote_ep) { voted = false; t_idle = now; }
        } else if (now - t_idle > a.idle_ticks) {
          uint32_t r = 0, ep = 0;
          if (lane == 0) r = serve_vote(a.state, gridDim.x, &ep);
          r = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)r);
          ep = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)ep);
          if (r == 0) break;
          if (r == 2) {  // unanimous: tell the host this launch left and the last message it saw
            if (lane == 0)
              __hip_atomic_store(&box->left, ((uint64_t)a.launch_id << 32) | (uint32_t)seq, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
            break;
          }
          voted = true;
          vote_ep = ep;
        }
#ifdef KSIM_STAMPS
        ++n_polls;
#endif
        __builtin_amdgcn_s_sleep(1);
      }
      if (got) {  // (an EXIT too: it may carry the decision on a tentative commit)
        s_msg[2 * lane] = q.x;
        s_msg[2 * lane + 1] = q.z;
      }
      if (type == KSIM_SERVE_SCHEDULE || type == KSIM_SERVE_ASSUME || type == KSIM_SERVE_UNDO) {
        // the payload through LDS: the pod into s_P, ports / scalars into this block's staging
        // slot (the evaluation reads them there)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        constexpr int PW = (int)(sizeof(ksim_pod) / 4);
        constexpr int XW = (int)(sizeof(ksim_scalar_req) / 4);
        int32_t* dst = reinterpret_cast<int32_t*>(&s_P);
        if (lane < PW) dst[lane] = (int32_t)s_msg[KSIM_SERVE_W_POD + lane];
        const int32_t np = (int32_t)s_msg[KSIM_SERVE_W_POD + offsetof(ksim_pod, port_cnt) / 4];
        const int32_t ns = (int32_t)s_msg[KSIM_SERVE_W_POD + offsetof(ksim_pod, scalar_cnt) / 4];
        int32_t* qp = reinterpret_cast<int32_t*>(pod_ports);
        int32_t* qs = reinterpret_cast<int32_t*>(pod_scalars);
        if (lane < 2 * np) qp[lane] = (int32_t)s_msg[KSIM_SERVE_W_PORTS + lane];  // (np <= KSIM_ONE_PORTS = 16)
        for (int k = lane; k < XW * ns; k += 64) qs[k] = (int32_t)s_msg[KSIM_SERVE_W_SCALARS + k];
        const int32_t sy = (int32_t)s_msg[KSIM_SERVE_W_SYNC];
        // the previous message committed counts other blocks read (affinity / volumes): acquire them
        if (sy & KSIM_SERVE_SYNC_ACQUIRE) __atomic_thread_fence(__ATOMIC_ACQUIRE);
        // the staging stores (and the last commit's) are acknowledged before the barrier below; the
        // CU's L1 needs no invalidation for them: every reader of a block's rows and staging slot is
        // a wave of the same workgroup, i.e. on the same CU (workgroup-scope coherence, KSIM_SERVE_L1INV
        // builds add the invalidation back for comparison)
#ifdef KSIM_SERVE_L1INV
        asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc0\n\ts_waitcnt vmcnt(0)" ::: "memory");
#else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
          s_P.port_off = me * KSIM_ONE_PORTS;
          s_P.scalar_off = me * KSIM_MAX_SCALAR;
          s_nc = (int32_t)s_msg[KSIM_SERVE_W_NOCOMMIT];
          s_tag = s_msg[KSIM_SERVE_W_TAG];
          s_node = (int64_t)(((uint64_t)s_msg[KSIM_SERVE_W_NODE + 1] << 32) | s_msg[KSIM_SERVE_W_NODE]);
        }
      }
      if (lane == 0) { s_type = type; s_got = got ? 1 : 0; s_undid = 0; }
    }
    __syncthreads();
#ifdef KSIM_STAMPS
    if (tid == 0) s_st[1] = __builtin_amdgcn_s_memrealtime();
#endif
    const int32_t type = s_type;
    // the host's decision on this block's tentative commit, before anything else reads the row
    if (s_got && s_tent.valid && s_msg[KSIM_SERVE_W_TENT_SEQ] == s_tent.seq && s_msg[KSIM_SERVE_W_TENT_ACT] != KSIM_TENT_NONE) {
      const bool undo = s_msg[KSIM_SERVE_W_TENT_ACT] == KSIM_TENT_UNDO;
      if (undo && wv == 0) {  // (shared state — mounts, affinity counts — only on an UNDO message: see ksim_common.h)
        if (lane == 0) {
          ksim_undo_commit(c, s_tent);
          if (ksim_is_vol_pod(c, s_tent.P)) ksim_vol_commit_body(*c.vol, s_tent.P, s_tent.node, -1, c.err);
        }
        if (ksim_is_aff_pod(c, s_tent.P)) ksim_aff_commit_body(*c.aff, s_tent.P, s_tent.node, -1, lane, 64);
        if (lane == 0) {
          s_undid = 1;
          __hip_atomic_store(&box->undo_ack, (uint64_t)s_tent.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
      __syncthreads();
      if (undo) ksim_row_cache_reload<NPT>(c, rcache, base, s_tent.node);
      __syncthreads();
      if (tid == 0) s_tent.valid = 0;
    }
    if (type != KSIM_SERVE_EXIT) seq = s_seq;
    if (type == KSIM_SERVE_SCHEDULE) {
      const ksim_pod P = s_P;
      ksim_pick_body<NPT, AUX>(c, P, 0, s_tag, s_nc, c.pick + (s_tag & 1u) * KSIM_PICK_WORDS, &s_keep, box->ans, seq, &s_tent,
                          &rcache, stamp);
    } else if (type == KSIM_SERVE_ASSUME) {
      // a resource delta onto a given node (ksim_pod_add): the block whose chunk holds it answers
      const int64_t node = s_node;
      if (node >= (int64_t)me * c.chunk && node < (int64_t)(me + 1) * c.chunk && wv == 0) {
        const ksim_pod P = s_P;
        const int32_t st = __shfl(ksim_commit_wave(c, P, node, lane), 0, 64);
        if (lane == 0 && ksim_is_vol_pod(c, P)) ksim_vol_commit_body(*c.vol, P, node, 1, c.err);
        if (ksim_is_aff_pod(c, P)) {
          if (lane == 0) ksim_svc_commit(*c.aff, P, node);
          ksim_aff_commit_body(*c.aff, P, node, 1, lane, 64);
        }
        // shared counts / mounts: released before the answer (the next message acquires them)
        if (ksim_is_aff_pod(c, P) || ksim_is_vol_pod(c, P)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        pk_answer(box->ans, seq, lane, (int32_t)node, 0, st, __hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                  s_keep, 0);
      }
      // the committed row's register copy: wave 0's stores, then the thread that caches the row
      __syncthreads();
      ksim_row_cache_reload<NPT>(c, rcache, base, s_node);
    } else if (type == KSIM_SERVE_UNDO) {
      // the explicit undo of a tentative commit of shared state: applied above by the block that
      // holds the record; the block owning the node answers (status 1: undone here, 0: no record
      // here — a relaunched kernel — and the host undoes it by a launch)
      const int64_t node = s_node;
      if (node >= (int64_t)me * c.chunk && node < (int64_t)(me + 1) * c.chunk && wv == 0) {
        if (s_undid) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // (the next message acquires)
        pk_answer(box->ans, seq, lane, (int32_t)node, 0, s_undid ? 1 : 0,
                  __hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), s_keep, 0);
      }
    } else {
      break;  // an exit message, or the grid left by the idle vote
    }
    __syncthreads();  // (the next poll overwrites the block's staging slot and s_P)
    t_idle = __builtin_amdgcn_s_memrealtime();
#ifdef KSIM_STAMPS
    if (tid == 0) {
      if (s_st[0]) { s_sum[0] += s_st[0] - t_end; s_cnt[0] += 1; }
      uint64_t prev = s_st[0];
      s_sum[11] += n_polls;
      s_cnt[11] += 1;
      n_polls = 0;
      for (int k = 1; k < 11; ++k) {
        if (s_st[k] && prev) { s_sum[k] += s_st[k] - prev; s_cnt[k] += 1; }
        if (s_st[k]) prev = s_st[k];
        s_st[k] = 0;
      }
      s_st[0] = 0;
      t_end = __builtin_amdgcn_s_memrealtime();
    }
#endif
  }
  // lastNodeIndex for the other forms (every block holds the same value): one writer, system scope
  if (me == 0 && tid == 0) __hip_atomic_store(c.counter, s_keep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#ifdef KSIM_STAMPS
  if (tid < 12) {
    atomicAdd((unsigned long long*)&c.dbg[64 + tid], (unsigned long long)s_sum[tid]);
    atomicAdd((unsigned long long*)&c.dbg[80 + tid], (unsigned long long)s_cnt[tid]);
  }
#endif
}

// Per-node evaluation of one pod without commit (ksim_evaluate).
__global__ __launch_bounds__(KSIM_BLOCK) void ksim_eval_kernel(KsimCtx c, int64_t pod, uint8_t* fit, uint32_t* reasons,
                                                             int64_t* score, uint8_t* rcls) {
  const int64_t i = (int64_t)blockIdx.x * KSIM_BLOCK + threadIdx.x;
  if (i >= c.n) return;
  ksim_pod P;  // (a branch, not a pointer select: the pod stays in registers)
  if (c.one) P = c.one_pod;
  else P = c.pods[pod];
  const int k1 = (c.w[KSIM_W_TAINT_TOLERATION] != 0) ? c.n_tt[P.cls] : 1;
  const int k2 = c.use_na ? c.n_na[P.cls] : 1;
  const KsimRow r = ksim_load_row(c, i);
  const uint32_t m = ksim_predicates(c, P, i, r);
  fit[i] = m == 0;
  reasons[i] = m;
  score[i] = ksim_map_score(c, P, r);
  rcls[i] = (uint8_t)((k1 * k2 > 1) ? ksim_rclass(c, P, i, k1, k2) : 0);
}

// Commit one pod to one node (ksim_assume, ksim_pod_add); status |= ksim_row_status.
// status[0] |= ksim_row_status, status[1] = the error word afterwards (KSIM_RES_STATUS / _ERR).
__global__ void ksim_assume_kernel(KsimCtx c, int64_t pod, int64_t node, int32_t* status) {
  if (blockIdx.x != 0 || threadIdx.x >= 64) return;
  ksim_pod P;  // (a branch, not a pointer select: the pod stays in registers)
  if (c.one) P = c.one_pod;
  else P = c.pods[pod];
  const int32_t st = ksim_commit_wave(c, P, node, threadIdx.x);
  if (threadIdx.x == 0) {
    if (ksim_is_vol_pod(c, P)) ksim_vol_commit_body(*c.vol, P, node, 1, c.err);
    *status |= st;
  }
  if (ksim_is_aff_pod(c, P)) {
    if (threadIdx.x == 0) ksim_svc_commit(*c.aff, P, node);
    ksim_aff_commit_body(*c.aff, P, node, 1, threadIdx.x, 64);
  }
  __syncthreads();
  if (threadIdx.x == 0) status[KSIM_RES_ERR - KSIM_RES_STATUS] = __hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Launch-mode entry points used by the host runtime (ksim_runtime.cpp).
extern "C" hipError_t ksim_launch_scan(const KsimCtx* c, int npt, int collect, int grid, hipStream_t s) {
#define KSIM_L(N, C) hipLaunchKernelGGL((ksim_scan_kernel<N, C>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c)
  if (collect) {
    switch (npt) {
      case 1: KSIM_L(1, true); break;
      case 2: KSIM_L(2, true); break;
      case 4: KSIM_L(4, true); break;
      default: KSIM_L(8, true); break;
    }
  } else {
    switch (npt) {
      case 1: KSIM_L(1, false); break;
      case 2: KSIM_L(2, false); break;
      case 4: KSIM_L(4, false); break;
      default: KSIM_L(8, false); break;
    }
  }
#undef KSIM_L
  return hipGetLastError();
}

// Whether the scan grid is co-resident (the fused pass A's grid barrier needs it).
// ksim_schedule_one on a cluster of n nodes in one workgroup (ksim_one_kernel): nodes per thread
// (0: more than 16 x 512 nodes), and the launch.
extern "C" int ksim_one_npt(int64_t n) {
  for (int npt : {2, 4, 6, 8, 10, 12, 16})
    if (n <= (int64_t)npt * ONE_BLOCK) return npt;
  return 0;
}
extern "C" hipError_t ksim_launch_one(const KsimCtx* c, int npt, hipStream_t s) {
#define KSIM_O(N) hipLaunchKernelGGL((ksim_one_kernel<N>), dim3(1), dim3(ONE_BLOCK), 0, s, *c)
  switch (npt) {
    case 2: KSIM_O(2); break;
    case 4: KSIM_O(4); break;
    case 6: KSIM_O(6); break;
    case 8: KSIM_O(8); break;
    case 10: KSIM_O(10); break;
    case 12: KSIM_O(12); break;
    case 16: KSIM_O(16); break;
    default: return hipErrorInvalidValue;
  }
#undef KSIM_O
  return hipGetLastError();
}

extern "C" int ksim_scan_coresident(int npt, int collect, int grid) {
#define KSIM_C(N, C) (ksim_check_coresident(ksim_scan_kernel<N, C>, grid, KSIM_BLOCK, 0) == hipSuccess)
  switch (npt) {
    case 1: return collect ? KSIM_C(1, true) : KSIM_C(1, false);
    case 2: return collect ? KSIM_C(2, true) : KSIM_C(2, false);
    case 4: return collect ? KSIM_C(4, true) : KSIM_C(4, false);
    default: return collect ? KSIM_C(8, true) : KSIM_C(8, false);
  }
#undef KSIM_C
}

extern "C" hipError_t ksim_launch_ipa_pass(const KsimCtx* c, int npt, int grid, hipStream_t s) {
  switch (npt) {
    case 1: hipLaunchKernelGGL((ksim_ipa_pass_kernel<1>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c); break;
    case 2: hipLaunchKernelGGL((ksim_ipa_pass_kernel<2>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c); break;
    case 4: hipLaunchKernelGGL((ksim_ipa_pass_kernel<4>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c); break;
    default: hipLaunchKernelGGL((ksim_ipa_pass_kernel<8>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c); break;
  }
  return hipGetLastError();
}

extern "C" hipError_t ksim_launch_eval(const KsimCtx* c, int64_t pod, uint8_t* fit, uint32_t* reasons, int64_t* score,
                                       uint8_t* rcls, hipStream_t s) {
  const int grid = (int)((c->n + KSIM_BLOCK - 1) / KSIM_BLOCK);
  hipLaunchKernelGGL(ksim_eval_kernel, dim3(grid), dim3(KSIM_BLOCK), 0, s, *c, pod, fit, reasons, score, rcls);
  return hipGetLastError();
}

extern "C" hipError_t ksim_launch_assume(const KsimCtx* c, int64_t pod, int64_t node, int32_t* status, hipStream_t s) {
  hipLaunchKernelGGL(ksim_assume_kernel, dim3(1), dim3(64), 0, s, *c, pod, node, status);
  return hipGetLastError();
}

// per-pod pick kernel: <= KSIM_PICK_MAXG blocks of KSIM_BLOCK threads, npt nodes per thread
extern "C" int ksim_pick_coresident(int npt, int grid) {
  hipError_t e = hipErrorInvalidValue;
  switch (npt) {
    case 1: e = (ksim_check_coresident(ksim_pick_kernel<1, false>, grid, KSIM_BLOCK, 0) == hipSuccess ? ksim_check_coresident(ksim_pick_kernel<1, true>, grid, KSIM_BLOCK, 0) : hipErrorInvalidValue); break;
    case 2: e = (ksim_check_coresident(ksim_pick_kernel<2, false>, grid, KSIM_BLOCK, 0) == hipSuccess ? ksim_check_coresident(ksim_pick_kernel<2, true>, grid, KSIM_BLOCK, 0) : hipErrorInvalidValue); break;
    case 4: e = (ksim_check_coresident(ksim_pick_kernel<4, false>, grid, KSIM_BLOCK, 0) == hipSuccess ? ksim_check_coresident(ksim_pick_kernel<4, true>, grid, KSIM_BLOCK, 0) : hipErrorInvalidValue); break;
    case 8: e = (ksim_check_coresident(ksim_pick_kernel<8, false>, grid, KSIM_BLOCK, 0) == hipSuccess ? ksim_check_coresident(ksim_pick_kernel<8, true>, grid, KSIM_BLOCK, 0) : hipErrorInvalidValue); break;
  }
  return e == hipSuccess ? 1 : 0;
}

extern "C" int ksim_serve_coresident(int npt, int grid) {
  hipError_t e = hipErrorInvalidValue;
  switch (npt) {
    case 1: e = (ksim_check_coresident(ksim_serve_kernel<1, false>, grid, KSIM_BLOCK, 0) == hipSuccess ? ksim_check_coresident(ksim_serve_kernel<1, true>, grid, KSIM_BLOCK, 0) : hipErrorInvalidValue); break;
    case 2: e = (ksim_check_coresident(ksim_serve_kernel<2, false>, grid, KSIM_BLOCK, 0) == hipSuccess ? ksim_check_coresident(ksim_serve_kernel<2, true>, grid, KSIM_BLOCK, 0) : hipErrorInvalidValue); break;
    case 4: e = (ksim_check_coresident(ksim_serve_kernel<4, false>, grid, KSIM_BLOCK, 0) == hipSuccess ? ksim_check_coresident(ksim_serve_kernel<4, true>, grid, KSIM_BLOCK, 0) : hipErrorInvalidValue); break;
    case 8: e = (ksim_check_coresident(ksim_serve_kernel<8, false>, grid, KSIM_BLOCK, 0) == hipSuccess ? ksim_check_coresident(ksim_serve_kernel<8, true>, grid, KSIM_BLOCK, 0) : hipErrorInvalidValue); break;
  }
  return e == hipSuccess ? 1 : 0;
}

extern "C" hipError_t ksim_launch_serve(const KsimCtx* c, const KsimServeArgs* a, int npt, int grid, int aux, hipStream_t s) {
  if (grid <= 0 || grid > KSIM_PICK_MAXG || !c->pick || !a->box || !a->state || c->one) return hipErrorInvalidValue;
  switch (npt) {
    case 1:
      if (aux) hipLaunchKernelGGL((ksim_serve_kernel<1, true>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c, *a);
      else hipLaunchKernelGGL((ksim_serve_kernel<1, false>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c, *a);
      break;
    case 2:
      if (aux) hipLaunchKernelGGL((ksim_serve_kernel<2, true>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c, *a);
      else hipLaunchKernelGGL((ksim_serve_kernel<2, false>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c, *a);
      break;
    case 4:
      if (aux) hipLaunchKernelGGL((ksim_serve_kernel<4, true>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c, *a);
      else hipLaunchKernelGGL((ksim_serve_kernel<4, false>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c, *a);
      break;
    case 8:
      if (aux) hipLaunchKernelGGL((ksim_serve_kernel<8, true>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c, *a);
      else hipLaunchKernelGGL((ksim_serve_kernel<8, false>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c, *a);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" hipError_t ksim_launch_pick(const KsimCtx* c, int npt, int grid, int aux, hipStream_t s) {
  if (grid <= 0 || grid > KSIM_PICK_MAXG || !c->pick) return hipErrorInvalidValue;
  switch (npt) {
    case 1:
      if (aux) hipLaunchKernelGGL((ksim_pick_kernel<1, true>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c);
      else hipLaunchKernelGGL((ksim_pick_kernel<1, false>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c);
      break;
    case 2:
      if (aux) hipLaunchKernelGGL((ksim_pick_kernel<2, true>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c);
      else hipLaunchKernelGGL((ksim_pick_kernel<2, false>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c);
      break;
    case 4:
      if (aux) hipLaunchKernelGGL((ksim_pick_kernel<4, true>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c);
      else hipLaunchKernelGGL((ksim_pick_kernel<4, false>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c);
      break;
    case 8:
      if (aux) hipLaunchKernelGGL((ksim_pick_kernel<8, true>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c);
      else hipLaunchKernelGGL((ksim_pick_kernel<8, false>), dim3(grid), dim3(KSIM_BLOCK), 0, s, *c);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
