/*
 * ORACLE — test infrastructure only (the CPU baseline leg of bench.py and the large parity
 * tests load it through ctypes; the product never links it).
 *
 * cpu_ref.c — plain-C restatement of the vendored kube-scheduler v1.10 per-pod cycle at
 * the node-table level: the same struct-of-arrays node table, pod descriptors and
 * per-pod-class tables the product's host ingest produces (include/ksim.h), so it checks
 * the HIP kernels on million-pod workloads where the object-level Python oracle
 * (oracle/ksim_ref.py) is too slow.  The string semantics (labels, tolerations) are pinned
 * separately by ksim_ref.py against the reference's golden vectors.
 *
 * Per pod, exactly as the reference (paths under vendor/k8s.io/kubernetes/pkg/scheduler/):
 *   findNodesThatFit   core/generic_scheduler.go:289-378, podFitsOnNode :420-534,
 *                      predicatesOrdering algorithm/predicates/predicates.go:129-138
 *   FitError           core/generic_scheduler.go:72-90 (reason histogram)
 *   single fit         core/generic_scheduler.go:153-156 (no selectHost, no counter bump)
 *   PrioritizeNodes    core/generic_scheduler.go:542-676 (map, reduce, weighted sum)
 *   selectHost         core/generic_scheduler.go:183-198 + api/types.go:272-277
 *   assume / AddPod    scheduler.go:366, schedulercache/node_info.go:318-341
 * selectHost sorts the HostPriorityList descending by (score, host); with unique hosts that
 * order is total, so the (lastNodeIndex % C)-th entry among the C max-score hosts is found
 * here by one descending walk instead of an O(F log F) sort (same result, faster baseline).
 *
 * Compile: see oracle/Makefile (-O2 -ffp-contract=off -fno-fast-math, OpenMP for the
 * node-parallel fan-out that mirrors workqueue.Parallelize(16, ...)).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ksim.h"

typedef struct {
  int64_t n;
  int32_t n_scalar, port_slots;
  const int64_t *alloc_cpu, *alloc_mem, *alloc_gpu, *alloc_eph, *alloc_scalar;
  const int32_t *allowed_pods, *label_set, *taint_set;
  const uint32_t* cond;                       /* static condition flags */
  int64_t *req_cpu, *req_mem, *req_gpu, *req_eph, *nz_cpu, *nz_mem, *req_scalar;
  int32_t* pod_count;
  uint64_t* ports;                            /* [port_slots][n] */
  int32_t* port_count;
} RefNodes;

/* ---- priorities: least_requested.go:44-53, most_requested.go:45-55,
 *      balanced_resource_allocation.go:39-61 (Go int64 truncation, IEEE f64) ---- */
static int64_t least_score(int64_t req, int64_t cap) {
  if (cap == 0 || req > cap) return 0;
  return (int64_t)((uint64_t)(cap - req) * 10u) / cap;
}
static int64_t most_score(int64_t req, int64_t cap) {
  if (cap == 0 || req > cap) return 0;
  return (int64_t)((uint64_t)req * 10u) / cap;
}
static double fraction(int64_t req, int64_t cap) { return cap == 0 ? 1.0 : (double)req / (double)cap; }
static int64_t balanced_score(int64_t rc, int64_t cc, int64_t rm, int64_t cm) {
  double fc = fraction(rc, cc), fm = fraction(rm, cm);
  if (fc >= 1 || fm >= 1) return 0;
  double diff = fabs(fc - fm);
  return (int64_t)((1 - diff) * 10.0);
}
/* reduce.go:29-64 for one value */
static int64_t normalize(int64_t v, int64_t mx, int reverse) {
  if (mx == 0) return reverse ? 10 : v;
  int64_t s = (int64_t)((uint64_t)10 * (uint64_t)v) / mx;
  return reverse ? 10 - s : s;
}

static int bit(const uint32_t* tab, int64_t row, int64_t words, int32_t idx) {
  return (int)((tab[row * words + (idx >> 5)] >> (idx & 31)) & 1u);
}

/* HostPortInfo.CheckConflict (util/utils.go:101-130) */
static int port_conflict(const RefNodes* N, int64_t i, uint64_t want) {
  uint32_t wip = (uint32_t)(want >> 40);
  for (int32_t s = 0; s < N->port_count[i]; ++s) {
    uint64_t e = N->ports[(int64_t)s * N->n + i];
    if ((e & 0xFFFFFFFFFFull) != (want & 0xFFFFFFFFFFull)) continue;
    uint32_t eip = (uint32_t)(e >> 40);
    if (wip == 0 || eip == 0 || eip == wip) return 1;
  }
  return 0;
}

/* PodFitsResources (predicates.go:706-778) */
static uint32_t pred_resources(const RefNodes* N, const ksim_pod* P, const ksim_scalar_req* sc, int64_t i) {
  uint32_t m = 0;
  if (N->pod_count[i] + 1 > N->allowed_pods[i]) m |= 1u << KSIM_R_INSUFFICIENT_PODS;
  if (!(P->flags & KSIM_POD_ANY_REQUEST)) return m;
  if (N->alloc_cpu[i] < P->req_cpu + N->req_cpu[i]) m |= 1u << KSIM_R_INSUFFICIENT_CPU;
  if (N->alloc_mem[i] < P->req_mem + N->req_mem[i]) m |= 1u << KSIM_R_INSUFFICIENT_MEMORY;
  if (N->alloc_gpu[i] < P->req_gpu + N->req_gpu[i]) m |= 1u << KSIM_R_INSUFFICIENT_GPU;
  if (N->alloc_eph[i] < P->req_eph + N->req_eph[i]) m |= 1u << KSIM_R_INSUFFICIENT_EPHEMERAL;
  for (int32_t s = 0; s < P->scalar_cnt; ++s) {
    const ksim_scalar_req* q = &sc[P->scalar_off + s];
    int64_t off = (int64_t)q->col * N->n + i;
    if (N->alloc_scalar[off] < q->req + N->req_scalar[off]) m |= 1u << (KSIM_R_INSUFFICIENT_SCALAR0 + q->col);
  }
  return m;
}

static uint32_t pred_host(const ksim_pod* P, int64_t i) {
  return (P->host == -1 || P->host == i) ? 0u : (1u << KSIM_R_HOSTNAME);
}

static uint32_t pred_ports(const RefNodes* N, const ksim_pod* P, const uint64_t* pp, int64_t i) {
  for (int32_t k = 0; k < P->port_cnt; ++k)
    if (port_conflict(N, i, pp[P->port_off + k])) return 1u << KSIM_R_HOST_PORTS;
  return 0;
}

typedef struct {
  const ksim_class_tables* T;
  int64_t lw, tw;
} RefTables;

static uint32_t pred_selector(const RefNodes* N, const RefTables* T, const ksim_pod* P, int64_t i) {
  return bit(T->T->sel_ok, P->cls, T->lw, N->label_set[i]) ? 0u : (1u << KSIM_R_NODE_SELECTOR);
}

/* podFitsOnNode: the reasons of the first failing predicate in predicatesOrdering */
static uint32_t pod_fits_on_node(uint32_t preds, const RefNodes* N, const RefTables* T, const ksim_pod* P,
                                 const uint64_t* pp, const ksim_scalar_req* sc, int64_t i) {
  uint32_t fl = N->cond[i], m;
  if (preds & KSIM_P_CHECK_NODE_CONDITION) {
    m = fl & (KSIM_N_NOT_READY | KSIM_N_OUT_OF_DISK | KSIM_N_NET_UNAVAIL | KSIM_N_UNSCHEDULABLE);
    if (m) return m;
  }
  if ((preds & KSIM_P_CHECK_NODE_UNSCHEDULABLE) && (fl & KSIM_N_UNSCHEDULABLE)) return 1u << KSIM_R_UNSCHEDULABLE;
  if (preds & KSIM_P_GENERAL) {  /* predicates.go:1059-1120: all four run */
    m = pred_resources(N, P, sc, i) | pred_host(P, i) | pred_ports(N, P, pp, i) | pred_selector(N, T, P, i);
    if (m) return m;
  }
  if ((preds & KSIM_P_HOSTNAME) && (m = pred_host(P, i))) return m;
  if ((preds & KSIM_P_HOST_PORTS) && (m = pred_ports(N, P, pp, i))) return m;
  if ((preds & KSIM_P_NODE_SELECTOR) && (m = pred_selector(N, T, P, i))) return m;
  if ((preds & KSIM_P_RESOURCES) && (m = pred_resources(N, P, sc, i))) return m;
  if ((preds & KSIM_P_TAINTS) && !bit(T->T->taint_ok, P->cls, T->tw, N->taint_set[i])) return 1u << KSIM_R_TAINTS;
  if ((preds & KSIM_P_NOEXEC_TAINTS) && !bit(T->T->noexec_ok, P->cls, T->tw, N->taint_set[i])) return 1u << KSIM_R_TAINTS;
  if ((preds & KSIM_P_LABEL_PRESENCE) && (fl & KSIM_N_LABEL_PRESENCE)) return 1u << KSIM_R_LABEL_PRESENCE;
  if ((preds & KSIM_P_MEM_PRESSURE) && (P->flags & KSIM_POD_BEST_EFFORT) && (fl & KSIM_N_MEM_PRESSURE))
    return 1u << KSIM_R_MEM_PRESSURE;
  if ((preds & KSIM_P_DISK_PRESSURE) && (fl & KSIM_N_DISK_PRESSURE)) return 1u << KSIM_R_DISK_PRESSURE;
  return 0;
}

/* NodeInfo.AddPod + HostPortInfo.Add */
static int assume_pod(RefNodes* N, const ksim_pod* P, const uint64_t* pp, const ksim_scalar_req* sc, int64_t w) {
  N->req_cpu[w] += P->add_cpu;
  N->req_mem[w] += P->add_mem;
  N->req_gpu[w] += P->add_gpu;
  N->req_eph[w] += P->add_eph;
  N->nz_cpu[w] += P->nz_cpu;
  N->nz_mem[w] += P->nz_mem;
  N->pod_count[w] += 1;
  for (int32_t s = 0; s < P->scalar_cnt; ++s) {
    const ksim_scalar_req* q = &sc[P->scalar_off + s];
    N->req_scalar[(int64_t)q->col * N->n + w] += q->add;
  }
  for (int32_t k = 0; k < P->port_cnt; ++k) {
    uint64_t key = pp[P->port_off + k];
    int dup = 0;
    for (int32_t s = 0; s < N->port_count[w]; ++s)
      if (N->ports[(int64_t)s * N->n + w] == key) dup = 1;
    if (dup) continue;
    if (N->port_count[w] >= N->port_slots) return KSIM_E_OVERFLOW;
    N->ports[(int64_t)N->port_count[w] * N->n + w] = key;
    N->port_count[w] += 1;
  }
  return KSIM_OK;
}

/*
 * Runs pods [first, first+count) in order against the MUTABLE node state `st` (dynamic
 * columns, updated in place) and the static columns of `tab`.  Returns KSIM_OK or an error.
 */
int ksim_ref_run(const ksim_config* cfg, const ksim_node_table* tab, ksim_node_state* st, const ksim_class_tables* ct,
                 const ksim_pod* pods, const uint64_t* pod_ports, const ksim_scalar_req* pod_scalars, int64_t first,
                 int64_t count, int threads, int32_t* out_node, int32_t* out_reasons, uint64_t* io_counter) {
  RefNodes N = {tab->n_nodes, tab->n_scalar, tab->port_slots, tab->alloc_cpu, tab->alloc_mem, tab->alloc_gpu,
                tab->alloc_eph, tab->alloc_scalar, tab->allowed_pods, tab->label_set, tab->taint_set, tab->flags,
                st->req_cpu, st->req_mem, st->req_gpu, st->req_eph, st->nz_cpu, st->nz_mem, st->req_scalar,
                st->pod_count, st->ports, st->port_count};
  RefTables T = {ct, (ct->n_label_sets + 31) / 32, (ct->n_taint_sets + 31) / 32};
  const int64_t n = N.n;
  uint32_t* mask = (uint32_t*)malloc(sizeof(uint32_t) * n);
  int64_t* score = (int64_t*)malloc(sizeof(int64_t) * n);
  int64_t* ttv = (int64_t*)malloc(sizeof(int64_t) * n);
  int64_t* nav = (int64_t*)malloc(sizeof(int64_t) * n);
  if (!mask || !score || !ttv || !nav) { free(mask); free(score); free(ttv); free(nav); return KSIM_E_NOMEM; }
  uint64_t counter = *io_counter;
  const uint32_t preds = cfg->predicates;
  const int64_t wl = cfg->weights[KSIM_W_LEAST_REQUESTED], wm = cfg->weights[KSIM_W_MOST_REQUESTED];
  const int64_t wb = cfg->weights[KSIM_W_BALANCED], wt = cfg->weights[KSIM_W_TAINT_TOLERATION];
  const int64_t wa = cfg->weights[KSIM_W_NODE_AFFINITY];
  int rc = KSIM_OK;
  if (threads < 1) threads = 1;

  for (int64_t k = first; k < first + count && rc == KSIM_OK; ++k) {
    const ksim_pod* P = &pods[k];
    const int64_t nzc = P->nz_cpu, nzm = P->nz_mem;
    const int64_t cls = P->cls;
    int64_t F = 0;
    int64_t mxT = 0, mxA = 0;
    /* findNodesThatFit + the map priorities over every node (workqueue.Parallelize) */
#pragma omp parallel for num_threads(threads) schedule(static) reduction(+ : F) reduction(max : mxT, mxA)
    for (int64_t i = 0; i < n; ++i) {
      uint32_t m = pod_fits_on_node(preds, &N, &T, P, pod_ports, pod_scalars, i);
      mask[i] = m;
      if (m) continue;
      F += 1;
      const int64_t rcpu = nzc + N.nz_cpu[i], rmem = nzm + N.nz_mem[i];
      uint64_t s = 0;
      if (wl) s += (uint64_t)wl * (uint64_t)((least_score(rcpu, N.alloc_cpu[i]) + least_score(rmem, N.alloc_mem[i])) / 2);
      if (wm) s += (uint64_t)wm * (uint64_t)((most_score(rcpu, N.alloc_cpu[i]) + most_score(rmem, N.alloc_mem[i])) / 2);
      if (wb) s += (uint64_t)wb * (uint64_t)balanced_score(rcpu, N.alloc_cpu[i], rmem, N.alloc_mem[i]);
      score[i] = (int64_t)s;
      if (wt) {
        int64_t v = ct->tt_val[cls * KSIM_MAX_RCLASS + ct->tt_class[cls * ct->n_taint_sets + N.taint_set[i]]];
        ttv[i] = v;
        if (v > mxT) mxT = v;
      }
      if (wa) {
        int64_t v = ct->na_val[cls * KSIM_MAX_RCLASS + ct->na_class[cls * ct->n_label_sets + N.label_set[i]]];
        nav[i] = v;
        if (v > mxA) mxA = v;
      }
    }
    int64_t winner = -1;
    if (F == 0) {
      if (out_reasons) {
        int32_t* h = &out_reasons[(k - first) * KSIM_NREASONS];
        for (int r = 0; r < KSIM_NREASONS; ++r) h[r] = 0;
        for (int64_t i = 0; i < n; ++i)
          for (int r = 0; r < KSIM_NREASONS; ++r) h[r] += (mask[i] >> r) & 1u;
      }
    } else if (F == 1) {
      for (int64_t i = 0; i < n; ++i)
        if (!mask[i]) { winner = i; break; }
    } else {
      /* reduce + weighted sum, then the max */
      int64_t M = INT64_MIN;
      for (int64_t i = 0; i < n; ++i) {
        if (mask[i]) continue;
        uint64_t t = (uint64_t)score[i];
        if (cfg->no_priorities) t = 0;
        if (wt) t += (uint64_t)wt * (uint64_t)normalize(ttv[i], mxT, 1);
        if (wa) t += (uint64_t)wa * (uint64_t)normalize(nav[i], mxA, 0);
        /* NodePreferAvoidPods (node_prefer_avoid_pods.go:32-68): its weighted map score rides the
           node's NodeAffinity class (ksim_class_tables.na_add) */
        if (ct->na_add)
          t += (uint64_t)ct->na_add[cls * KSIM_MAX_RCLASS + ct->na_class[cls * ct->n_label_sets + N.label_set[i]]];
        score[i] = (int64_t)t;
        if (score[i] > M) M = score[i];
      }
      int64_t C = 0;
      for (int64_t i = 0; i < n; ++i) C += (!mask[i] && score[i] == M);
      int64_t ix = (int64_t)(counter % (uint64_t)C);
      counter += 1;
      for (int64_t i = n - 1; i >= 0; --i) {   /* descending (score, name rank) */
        if (mask[i] || score[i] != M) continue;
        if (ix == 0) { winner = i; break; }
        --ix;
      }
    }
    out_node[k - first] = (int32_t)winner;
    if (winner >= 0) rc = assume_pod(&N, P, pod_ports, pod_scalars, winner);
  }
  *io_counter = counter;
  free(mask); free(score); free(ttv); free(nav);
  return rc;
}
