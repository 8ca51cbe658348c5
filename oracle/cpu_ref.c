/*
 * ORACLE — test infrastructure only (the CPU baseline leg of bench.py and the large parity
 * tests load it through ctypes; the product never links it).
 *
 * cpu_ref.c — plain-C restatement of the vendored kube-scheduler v1.10 per-pod cycle at
 * the node-table level: the same struct-of-arrays node table, pod descriptors, per-pod-class
 * tables and (optionally) inter-pod affinity / SelectorSpread / volume tables the product's host
 * ingest produces (include/ksim.h), so it checks the HIP kernels on workloads where the
 * object-level Python oracle (oracle/ksim_ref.py) is too slow.  The string semantics (labels,
 * tolerations, affinity terms, volume identities) are pinned separately: ksim_ref.py against the
 * reference's golden vectors, and this file against ksim_ref.py from the same Kubernetes objects
 * (tests/test_oracle_c.py, tests/test_oracle_scale.py).
 *
 * Per pod, exactly as the reference (paths under vendor/k8s.io/kubernetes/pkg/scheduler/):
 *   findNodesThatFit   core/generic_scheduler.go:289-378, podFitsOnNode :420-534,
 *                      predicatesOrdering algorithm/predicates/predicates.go:129-138
 *   volumes            NoDiskConflict predicates.go:220-285, MaxPDVolumeCountChecker :287-507,
 *                      VolumeZoneChecker :539-633
 *   CheckServiceAffinity predicates.go:940-1016 (per (pod class, label set) verdict)
 *   MatchInterPodAffinity predicates.go:1143-1450
 *   FitError           core/generic_scheduler.go:72-90 (reason histogram)
 *   single fit         core/generic_scheduler.go:153-156 (no selectHost, no counter bump)
 *   PrioritizeNodes    core/generic_scheduler.go:542-676 (map, reduce, weighted sum):
 *                      NormalizeReduce priorities/reduce.go:29-64, InterPodAffinityPriority
 *                      priorities/interpod_affinity.go:118-240, SelectorSpread
 *                      priorities/selector_spreading.go:66-174
 *   selectHost         core/generic_scheduler.go:183-198 + api/types.go:272-277
 *   assume / AddPod    scheduler.go:366, schedulercache/node_info.go:318-341
 * selectHost sorts the HostPriorityList descending by (score, host); with unique hosts that
 * order is total, so the (lastNodeIndex % C)-th entry among the C max-score hosts is found
 * here by one descending walk instead of an O(F log F) sort (same result, faster baseline).
 *
 * Threads: workqueue.Parallelize(16, N, checkNode) (client-go util/workqueue/parallelizer.go:29-52)
 * fans every pod's node loop out to 16 goroutines; here one OpenMP team lives for the whole call
 * and splits the nodes into contiguous per-thread ranges each pod (barriers between the phases,
 * no fork/join per pod), so the thread count scales the node loop only.
 *
 * Compile: see oracle/Makefile (-O2 -ffp-contract=off -fno-fast-math, OpenMP).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ksim.h"

/* row width of the per-class value arrays (ksim_class_tables.val_width, ABI 7; 0 = 16) */
#define VW(ct) ((int64_t)((ct)->val_width ? (ct)->val_width : KSIM_MAX_RCLASS))

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

/* Mutable state of the optional tables (copies the caller owns; updated by every commit). */
typedef struct {
  int32_t* cnt;       /* affinity counted pairs [cnt_len] */
  int64_t* carried;   /* affinity carried terms [carried_len] */
  uint64_t* vslots;   /* volume slots [vol_slots][n] */
  int32_t* vcount;    /* used volume slots per node [n] */
  uint32_t* svc_conflict; /* service-affinity disagreement bits [n_svc] */
  int32_t svc_err;        /* set when a pod read a disagreeing label: the run is refused */
  int32_t pad;
} ksim_ref_extra;

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
  const ksim_affinity_tables* A;  /* NULL: no inter-pod affinity / spread tables */
  const ksim_volume_tables* V;    /* NULL: no volume tables */
  ksim_ref_extra* X;
} RefTables;

static uint32_t pred_selector(const RefNodes* N, const RefTables* T, const ksim_pod* P, int64_t i) {
  return bit(T->T->sel_ok, P->cls, T->lw, N->label_set[i]) ? 0u : (1u << KSIM_R_NODE_SELECTOR);
}

/* ---- volumes (the tables of ksim/volumes.py: a key per volume identity, per node the mounted
 *      keys with read-write / read-only / via-PVC mount counts) ---- */
static int vol_find(const RefTables* T, int64_t i, int32_t key) {
  const ksim_volume_tables* V = T->V;
  for (int32_t s = 0; s < T->X->vcount[i]; ++s)
    if ((int32_t)(T->X->vslots[(int64_t)s * V->n_nodes + i] >> 32) == key) return s;
  return -1;
}

/* NoDiskConflict (predicates.go:276-285 over isVolumeConflict :220-265): GCE PD / ISCSI / RBD
 * conflict unless both mounts are read-only, EBS always conflicts; PVC mounts are not looked at. */
static uint32_t pred_disk_conflict(const RefTables* T, const ksim_pod* P, int64_t i) {
  const ksim_volume_tables* V = T->V;
  const int32_t* vc = V->vc + 2 * (int64_t)(P->vol_class - 1);
  for (int32_t j = vc[0]; j < vc[0] + vc[1]; ++j) {
    const ksim_vol_ref* r = &V->refs[j];
    if (!(r->flags & (KSIM_VOL_CONFLICT_ANY | KSIM_VOL_CONFLICT_RW))) continue;
    const int s = vol_find(T, i, r->key);
    if (s < 0) continue;
    const uint64_t w = T->X->vslots[(int64_t)s * V->n_nodes + i];
    const uint32_t rw = (uint32_t)(w & 0x7FFu), ro = (uint32_t)((w >> 11) & 0x7FFu);
    if ((r->flags & KSIM_VOL_CONFLICT_ANY) ? (rw + ro > 0) : (rw > 0)) return 1u << KSIM_R_DISK_CONFLICT;
  }
  return 0;
}

/* MaxPDVolumeCountChecker.predicate (predicates.go:415-456) for one filter: the node's distinct
 * volume ids of the filter's kind plus the pod's new ones not yet mounted, against the limit. */
static uint32_t pred_max_volumes(const RefTables* T, const ksim_pod* P, int64_t i, int filt_idx) {
  const ksim_volume_tables* V = T->V;
  const uint32_t f = 1u << filt_idx;
  if (!(V->vc_filter[P->vol_class - 1] & f)) return 0;  /* len(newVolumes) == 0 (:427-430) */
  int32_t have = 0, add = 0;
  for (int32_t s = 0; s < T->X->vcount[i]; ++s)
    if (V->key_filter[(int32_t)(T->X->vslots[(int64_t)s * V->n_nodes + i] >> 32)] & f) ++have;
  const int32_t* vc = V->vc + 2 * (int64_t)(P->vol_class - 1);
  for (int32_t j = vc[0]; j < vc[0] + vc[1]; ++j) {
    const ksim_vol_ref* r = &V->refs[j];
    if ((r->flags & KSIM_VOL_NEW) && (V->key_filter[r->key] & f) && vol_find(T, i, r->key) < 0) ++add;
  }
  return have + add > V->max_vols[filt_idx] ? (1u << KSIM_R_MAX_VOLUME_COUNT) : 0u;
}

/* ---- inter-pod affinity (the tables of ksim/affinity.py) ---- */
static int32_t aff_dom(const ksim_affinity_tables* A, int32_t key, int64_t i) { return A->dom[(int64_t)key * A->n_nodes + i]; }

static int pair_hit(const RefTables* T, int32_t pair, int64_t i) {
  const ksim_affinity_tables* A = T->A;
  const int32_t d = aff_dom(A, A->pair_key[pair], i);
  return d >= 0 && T->X->cnt[A->pair_off[pair] + d] > 0;
}

/* InterPodAffinityMatches (predicates.go:1143-1160): satisfiesExistingPodsAntiAffinity
 * (:1340-1379), then the pod's required affinity terms (anyPodMatchesPodAffinityTerm :1161-1194,
 * a term no placed pod matches is waived when the pod matches it itself, :1405-1424), then its
 * required anti-affinity terms (:1430-1441). */
static uint32_t pred_interpod(const RefTables* T, const ksim_pod* P, int64_t i) {
  const ksim_affinity_tables* A = T->A;
  const uint32_t base = 1u << KSIM_R_POD_AFFINITY;
  if (P->aff_ident > 0) {
    const uint64_t* mw = A->ident_anti + (int64_t)(P->aff_ident - 1) * A->carry_words;
    for (int32_t e = 0; e < A->n_carry; ++e) {
      if (!((mw[e >> 6] >> (e & 63)) & 1u)) continue;
      const int32_t d = aff_dom(A, A->carry_key[e], i);
      if (d >= 0 && T->X->carried[A->carry_off[e] + d] > 0) return base | (1u << KSIM_R_EXISTING_ANTI_AFFINITY);
    }
  }
  if (P->aff_class <= 0) return 0;
  const int32_t* ac = A->ac + 6 * (int64_t)(P->aff_class - 1);
  for (int32_t j = ac[0]; j < ac[0] + ac[1]; ++j) {
    const ksim_aff_term* t = &A->terms[j];
    const int match = aff_dom(A, t->gate_key, i) >= 0 && pair_hit(T, t->pair, i);
    if (t->kind == KSIM_AFF_REQ_AFFINITY) {
      if (!match && (!t->self_ok || pair_hit(T, t->exist_pair, i))) return base | (1u << KSIM_R_AFFINITY_RULES);
    } else if (match) {
      return base | (1u << KSIM_R_ANTI_AFFINITY_RULES);
    }
  }
  return 0;
}

/* Does the pod read InterPodAffinityPriority (own preferred terms, or carried priority terms of
 * placed pods it matches)?  Otherwise every count is 0 and the priority is 0 everywhere. */
static int interpod_prio_work(const ksim_affinity_tables* A, const ksim_pod* P) {
  if (P->aff_class > 0 && A->ac[6 * (int64_t)(P->aff_class - 1) + 3] > 0) return 1;
  if (P->aff_ident <= 0) return 0;
  const uint64_t* mw = A->ident_prio + (int64_t)(P->aff_ident - 1) * A->carry_words;
  for (int32_t w = 0; w < A->carry_words; ++w)
    if (mw[w]) return 1;
  return 0;
}

/* CalculateInterPodAffinityPriority's per-node count (interpod_affinity.go:124-214) before the
 * normalisation: the pod's preferred terms weight the placed pods they match in the node's
 * topology domain; the terms placed pods carry add their weights where the pod matches them. */
static int64_t interpod_raw(const RefTables* T, const ksim_pod* P, int64_t i) {
  const ksim_affinity_tables* A = T->A;
  int64_t s = 0;
  if (P->aff_class > 0) {
    const int32_t* ac = A->ac + 6 * (int64_t)(P->aff_class - 1);
    for (int32_t j = ac[2]; j < ac[2] + ac[3]; ++j) {
      const ksim_aff_term* t = &A->terms[j];
      const int32_t d = aff_dom(A, A->pair_key[t->pair], i);
      if (d >= 0) s += t->weight * (int64_t)T->X->cnt[A->pair_off[t->pair] + d];
    }
  }
  if (P->aff_ident > 0) {
    const uint64_t* mw = A->ident_prio + (int64_t)(P->aff_ident - 1) * A->carry_words;
    for (int32_t e = 0; e < A->n_carry; ++e) {
      if (!((mw[e >> 6] >> (e & 63)) & 1u)) continue;
      const int32_t d = aff_dom(A, A->carry_key[e], i);
      if (d >= 0) s += T->X->carried[A->carry_off[e] + d];
    }
  }
  return s;
}

/* podFitsOnNode: the reasons of the first failing predicate in predicatesOrdering */
/* CheckServiceAffinity with services (predicates.go:980-1011): the labels the pod's nodeSelector
 * leaves open take the values of the node of the first cached pod with the pod's labels
 * (serviceAffinityMetadataProducer :920-940 lists them in pod-lister order).  Over the counted
 * pairs of the class's service-affinity identity: with matching pods cached, a label some of their
 * nodes carry must have the value they all share; when their nodes disagree on an open label
 * (svc_conflict) the answer would depend on the lister's order and the run is refused. */
static uint32_t pred_svc_lender(const RefTables* T, const ksim_pod* P, int64_t i) {
  const ksim_affinity_tables* A = T->A;
  if (!A || !A->svc_class || P->aff_class <= 0) return 0;
  const int32_t v = A->svc_class[P->aff_class - 1];
  if (v < 0) return 0;
  const uint32_t open = A->svc_miss[P->aff_class - 1];
  const ksim_svc_ident* S = &A->svc_ident[v];
  const int32_t matching = T->X->cnt[A->pair_off[S->pair_all]];
  if (matching == 0) return 0;
  if (T->X->svc_conflict[v] & open) {
    __atomic_store_n(&T->X->svc_err, 1, __ATOMIC_RELAXED);
    return 1u << KSIM_R_SERVICE_AFFINITY;
  }
  for (int l = 0; l < A->n_svc_labels; ++l) {
    if (!((open >> l) & 1u) || T->X->cnt[A->pair_off[S->pair_present[l]]] == 0) continue;
    const int32_t pv = S->pair_value[l];
    const int32_t d = aff_dom(A, A->pair_key[pv], i);
    if (d < 0 || T->X->cnt[A->pair_off[pv] + d] != matching) return 1u << KSIM_R_SERVICE_AFFINITY;
  }
  return 0;
}

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
  const int vol = T->V && P->vol_class > 0;
  if ((preds & KSIM_P_DISK_CONFLICT) && vol && (m = pred_disk_conflict(T, P, i))) return m;
  if ((preds & KSIM_P_TAINTS) && !bit(T->T->taint_ok, P->cls, T->tw, N->taint_set[i])) return 1u << KSIM_R_TAINTS;
  if ((preds & KSIM_P_NOEXEC_TAINTS) && !bit(T->T->noexec_ok, P->cls, T->tw, N->taint_set[i])) return 1u << KSIM_R_TAINTS;
  if ((preds & KSIM_P_LABEL_PRESENCE) && (fl & KSIM_N_LABEL_PRESENCE)) return 1u << KSIM_R_LABEL_PRESENCE;
  if ((preds & KSIM_P_SERVICE_AFFINITY) && T->T->svc_ok && !bit(T->T->svc_ok, P->cls, T->lw, N->label_set[i]))
    return 1u << KSIM_R_SERVICE_AFFINITY;
  if ((preds & KSIM_P_SERVICE_AFFINITY) && (m = pred_svc_lender(T, P, i))) return m;
  if (vol) {
    static const uint32_t keys[3] = {KSIM_P_MAX_EBS, KSIM_P_MAX_GCE_PD, KSIM_P_MAX_AZURE_DISK};
    for (int t = 0; t < 3; ++t)
      if ((preds & keys[t]) && (m = pred_max_volumes(T, P, i, t))) return m;
    if ((preds & KSIM_P_VOLUME_ZONE) && T->V->zone_ok &&
        !bit(T->V->zone_ok, P->vol_class - 1, T->V->zone_words, N->label_set[i]))
      return 1u << KSIM_R_VOLUME_ZONE;
  }
  if ((preds & KSIM_P_MEM_PRESSURE) && (P->flags & KSIM_POD_BEST_EFFORT) && (fl & KSIM_N_MEM_PRESSURE))
    return 1u << KSIM_R_MEM_PRESSURE;
  if ((preds & KSIM_P_DISK_PRESSURE) && (fl & KSIM_N_DISK_PRESSURE)) return 1u << KSIM_R_DISK_PRESSURE;
  if ((preds & KSIM_P_INTERPOD_AFFINITY) && T->A && (P->aff_ident > 0 || P->aff_class > 0)) return pred_interpod(T, P, i);
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

/* NodeInfo.AddPod of the pod's volumes: one mount of each ref's key (read-write, read-only or via a
 * PVC) on node w. */
static int assume_volumes(RefTables* T, const ksim_pod* P, int64_t w) {
  const ksim_volume_tables* V = T->V;
  const int32_t* vc = V->vc + 2 * (int64_t)(P->vol_class - 1);
  for (int32_t j = vc[0]; j < vc[0] + vc[1]; ++j) {
    const ksim_vol_ref* r = &V->refs[j];
    const int sh = (r->flags & KSIM_VOL_VIA_PVC) ? 22 : (r->flags & KSIM_VOL_READ_ONLY) ? 11 : 0;
    const uint64_t fmask = (sh == 22 ? 0x3FFull : 0x7FFull) << sh, one = 1ull << sh;
    const int s = vol_find(T, w, r->key);
    if (s >= 0) {
      uint64_t* slot = &T->X->vslots[(int64_t)s * V->n_nodes + w];
      if ((*slot & fmask) == fmask) return KSIM_E_OVERFLOW;
      *slot += one;
    } else {
      const int32_t cnt = T->X->vcount[w];
      if (cnt >= V->vol_slots) return KSIM_E_OVERFLOW;
      T->X->vslots[(int64_t)cnt * V->n_nodes + w] = ((uint64_t)(uint32_t)r->key << 32) | one;
      T->X->vcount[w] = cnt + 1;
    }
  }
  return KSIM_OK;
}

/* NodeInfo.AddPod of an affinity pod: +1 on every counted pair whose selector its identity
 * matches (at node w's domain of the pair's key), + its carried amounts at w's domains. */
static void assume_affinity(RefTables* T, const ksim_pod* P, int64_t w) {
  const ksim_affinity_tables* A = T->A;
  if (A->svc_class && P->aff_ident > 0) {
    /* the service-affinity identities this pod's labels match: record the labels on which node w
       disagrees with their cached pods' nodes (before this pod counts) */
    for (int32_t e = A->svc_of_off[P->aff_ident - 1]; e < A->svc_of_off[P->aff_ident]; ++e) {
      const int32_t v = A->svc_of[e];
      const ksim_svc_ident* S = &A->svc_ident[v];
      const int32_t matching = T->X->cnt[A->pair_off[S->pair_all]];
      if (matching == 0) continue;
      for (int l = 0; l < A->n_svc_labels; ++l) {
        const int32_t pv = S->pair_value[l];
        const int32_t d = aff_dom(A, A->pair_key[pv], w);
        const int32_t same = d >= 0 ? T->X->cnt[A->pair_off[pv] + d] : matching - T->X->cnt[A->pair_off[S->pair_present[l]]];
        if (same != matching) T->X->svc_conflict[v] |= 1u << l;
      }
    }
  }
  if (P->aff_ident > 0) {
    const uint64_t* sm = A->ident_sel + (int64_t)(P->aff_ident - 1) * A->sel_words;
    for (int32_t c = 0; c < A->n_pair; ++c) {
      const int32_t s = A->pair_sel[c];
      if (!((sm[s >> 6] >> (s & 63)) & 1ull)) continue;
      const int32_t d = aff_dom(A, A->pair_key[c], w);
      if (d >= 0) T->X->cnt[A->pair_off[c] + d] += 1;
    }
  }
  if (P->aff_class > 0) {
    const int32_t* ac = A->ac + 6 * (int64_t)(P->aff_class - 1);
    for (int32_t j = ac[4]; j < ac[4] + ac[5]; ++j) {
      const ksim_aff_carry* k = &A->carries[j];
      const int32_t d = aff_dom(A, A->carry_key[k->term], w);
      if (d >= 0) T->X->carried[A->carry_off[k->term] + d] += k->amount;
    }
  }
}

/* CalculateSpreadPriorityReduce's score of one fit node (selector_spreading.go:121-174): float64
 * without contraction as in Go. */
static int64_t spread_score(int64_t cnt, int64_t max_node, int have_zones, int32_t zone, int64_t zone_cnt,
                            int64_t max_zone) {
  const double zw = 2.0 / 3.0; /* zoneWeighting (selector_spreading.go:33) */
  double f = 10.0;
  if (max_node > 0) f = 10.0 * ((double)(max_node - cnt) / (double)max_node);
  if (have_zones && zone >= 0) {
    double zs = 10.0;
    if (max_zone > 0) zs = 10.0 * ((double)(max_zone - zone_cnt) / (double)max_zone);
    f = (f * (1.0 - zw)) + (zw * zs);
  }
  return (int64_t)f;
}

/* The auxiliary priority's score of one fit node (ksim_affinity_tables.aux_*): KSIM_AUX_SPREAD is
 * spread_score over the aux pair and key; KSIM_AUX_SERVICE_ANTI is
 * CalculateAntiAffinityPriorityReduce (selector_spreading.go:248-275): 0 without the label, else
 * MaxPriority x (total - count of the node's label value) / total over the fit nodes (MaxPriority
 * when total is 0), float64 as in Go. */
static int64_t aux_score(int kind, int64_t cnt, int32_t d, int64_t dsum, int64_t amx, int64_t atot, int ahz,
                         int64_t azmx) {
  if (kind == KSIM_AUX_SPREAD) return spread_score(cnt, amx, ahz, d, dsum, azmx);
  if (d < 0) return 0;
  if (atot <= 0) return 10;
  return (int64_t)(10.0 * ((double)(atot - dsum) / (double)atot));
}

#define MAXT 256

/* Per-thread partials of one pod (one cache line apart). */
typedef struct {
  int64_t F, mxT, mxA, mn, mx, smx, hz;
  int64_t amx, atot, ahz;  /* the auxiliary priority (ksim_affinity_tables.aux_*) */
  int64_t M, C;
  int32_t hist[KSIM_NREASONS];
  char pad[64];
} RefPart;

/*
 * Runs pods [first, first+count) in order against the MUTABLE node state `st` (dynamic columns,
 * updated in place), the static columns of `tab`, and — when `at` / `vt` are given — the affinity
 * / volume tables with their mutable counts in `xs` (copies of at->cnt / carried, vt->slots /
 * slot_count the caller owns).  Returns KSIM_OK or an error.
 */
int ksim_ref_run_ex(const ksim_config* cfg, const ksim_node_table* tab, ksim_node_state* st, const ksim_class_tables* ct,
                    const ksim_affinity_tables* at, const ksim_volume_tables* vt, ksim_ref_extra* xs,
                    const ksim_pod* pods, const uint64_t* pod_ports, const ksim_scalar_req* pod_scalars, int64_t first,
                    int64_t count, int threads, int32_t* out_node, int32_t* out_reasons, uint64_t* io_counter) {
  RefNodes N = {tab->n_nodes, tab->n_scalar, tab->port_slots, tab->alloc_cpu, tab->alloc_mem, tab->alloc_gpu,
                tab->alloc_eph, tab->alloc_scalar, tab->allowed_pods, tab->label_set, tab->taint_set, tab->flags,
                st->req_cpu, st->req_mem, st->req_gpu, st->req_eph, st->nz_cpu, st->nz_mem, st->req_scalar,
                st->pod_count, st->ports, st->port_count};
  RefTables T = {ct, (ct->n_label_sets + 31) / 32, (ct->n_taint_sets + 31) / 32, at, vt, xs};
  if ((at || vt) && !xs) return KSIM_E_INVAL;
  const int64_t n = N.n;
  if (threads < 1) threads = 1;
  if (threads > MAXT) threads = MAXT;
  if ((int64_t)threads > n && n > 0) threads = (int)n;
  const int n_zone = (at && at->zone_key >= 0) ? at->n_dom[at->zone_key] : 0;
  uint32_t* mask = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  int64_t* score = (int64_t*)malloc(sizeof(int64_t) * (n ? n : 1));
  int64_t* ttv = (int64_t*)malloc(sizeof(int64_t) * (n ? n : 1));
  int64_t* nav = (int64_t*)malloc(sizeof(int64_t) * (n ? n : 1));
  int64_t* raw = (int64_t*)malloc(sizeof(int64_t) * (n ? n : 1));
  int64_t* zsum = (int64_t*)calloc((size_t)threads * (n_zone + 1), sizeof(int64_t));
  int64_t* zall = (int64_t*)calloc((size_t)n_zone + 1, sizeof(int64_t));
  RefPart* part = (RefPart*)calloc((size_t)threads, sizeof(RefPart));
  const int aux_on = at && at->aux_pair && at->aux_weight && !cfg->no_priorities;
  const int n_adom = aux_on ? at->n_dom[at->aux_key] : 0;
  int64_t* asum = (int64_t*)calloc((size_t)threads * (n_adom + 1), sizeof(int64_t));
  int64_t* aall = (int64_t*)calloc((size_t)n_adom + 1, sizeof(int64_t));
  if (!mask || !score || !ttv || !nav || !raw || !zsum || !zall || !part || !asum || !aall) {
    free(mask); free(score); free(ttv); free(nav); free(raw); free(zsum); free(zall); free(part); free(asum); free(aall);
    return KSIM_E_NOMEM;
  }
  uint64_t counter = *io_counter;
  const uint32_t preds = cfg->predicates;
  const int64_t wl = cfg->weights[KSIM_W_LEAST_REQUESTED], wm = cfg->weights[KSIM_W_MOST_REQUESTED];
  const int64_t wb = cfg->weights[KSIM_W_BALANCED], wt = cfg->weights[KSIM_W_TAINT_TOLERATION];
  const int64_t wa = cfg->weights[KSIM_W_NODE_AFFINITY];
  const int64_t wi = cfg->weights[KSIM_W_INTERPOD_AFFINITY], wsp = cfg->weights[KSIM_W_SELECTOR_SPREAD];
  int rc = KSIM_OK;
  /* the pod's decision, shared between the phases */
  int64_t winner = -1, M = 0, ixv = 0, G_zmx = 0, G_azmx = 0;

#pragma omp parallel num_threads(threads)
  {
    const int tn = omp_get_thread_num(), T_ = omp_get_num_threads();
    const int64_t lo = n * tn / T_, hi = n * (tn + 1) / T_;
    RefPart* my = &part[tn];
    int64_t* myz = zsum + (size_t)tn * (n_zone + 1);
    int64_t* mya = asum + (size_t)tn * (n_adom + 1);
    for (int64_t k = first; k < first + count; ++k) {
      if (rc != KSIM_OK) break;  /* uniform: read after the previous pod's last barrier */
      const ksim_pod* P = &pods[k];
      const int64_t nzc = P->nz_cpu, nzm = P->nz_mem;
      const int64_t cls = P->cls;
      const int ipa = at && wi && !cfg->no_priorities && interpod_prio_work(at, P);
      const int32_t sp = (at && wsp && !cfg->no_priorities && at->spread_pair && P->aff_class > 0)
                             ? at->spread_pair[P->aff_class - 1] : -1;
      const int32_t ap = (aux_on && P->aff_class > 0) ? at->aux_pair[P->aff_class - 1] : -1;
      const int aread = aux_on && (ap >= 0 || at->aux_kind == KSIM_AUX_SERVICE_ANTI);
      /* ---- phase 1: findNodesThatFit + the map priorities over this thread's nodes ---- */
      int64_t F = 0, mxT = 0, mxA = 0, mn = 0, mx = 0, smx = 0, hz = 0, amx = 0, atot = 0, ahz = 0;
      for (int z = 0; z < n_zone; ++z) myz[z] = 0;
      for (int z = 0; z < n_adom; ++z) mya[z] = 0;
      for (int64_t i = lo; i < hi; ++i) {
        const uint32_t m = pod_fits_on_node(preds, &N, &T, P, pod_ports, pod_scalars, i);
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
          int64_t v = ct->tt_val[cls * VW(ct) + ct->tt_class[cls * ct->n_taint_sets + N.taint_set[i]]];
          ttv[i] = v;
          if (v > mxT) mxT = v;
        }
        if (wa) {
          int64_t v = ct->na_val[cls * VW(ct) + ct->na_class[cls * ct->n_label_sets + N.label_set[i]]];
          nav[i] = v;
          if (v > mxA) mxA = v;
        }
        if (ipa) { /* the accumulators start at 0 (interpod_affinity.go:129-131, 218-226) */
          const int64_t r = interpod_raw(&T, P, i);
          raw[i] = r;
          if (r < mn) mn = r;
          if (r > mx) mx = r;
        }
        if (sp >= 0) { /* selector_spreading.go:125-145: maxCountByNodeName, countsByZone */
          const int64_t c = xs->cnt[at->pair_off[sp] + aff_dom(at, at->pair_key[sp], i)];
          if (c > smx) smx = c;
          const int32_t z = at->zone_key >= 0 ? aff_dom(at, at->zone_key, i) : -1;
          if (z >= 0) { hz = 1; myz[z] += c; }
        }
        if (ap >= 0) { /* the auxiliary pair: max, total, haveZones, per-domain sums */
          const int64_t c = xs->cnt[at->pair_off[ap] + aff_dom(at, at->pair_key[ap], i)];
          if (c > amx) amx = c;
          atot += c;
          const int32_t d = aff_dom(at, at->aux_key, i);
          if (d >= 0) { ahz = 1; mya[d] += c; }
        }
      }
      my->F = F; my->mxT = mxT; my->mxA = mxA; my->mn = mn; my->mx = mx; my->smx = smx; my->hz = hz;
      my->amx = amx; my->atot = atot; my->ahz = ahz;
#pragma omp barrier
      /* ---- combine (every thread, the same result): fit count and the reduce maxima ---- */
      int64_t Ft = 0, mT = 0, mA = 0, gmn = 0, gmx = 0, gsmx = 0, ghz = 0, gamx = 0, gatot = 0, gahz = 0;
      for (int t = 0; t < T_; ++t) {
        if (part[t].amx > gamx) gamx = part[t].amx;
        gatot += part[t].atot;
        if (part[t].ahz) gahz = 1;
        Ft += part[t].F;
        if (part[t].mxT > mT) mT = part[t].mxT;
        if (part[t].mxA > mA) mA = part[t].mxA;
        if (part[t].mn < gmn) gmn = part[t].mn;
        if (part[t].mx > gmx) gmx = part[t].mx;
        if (part[t].smx > gsmx) gsmx = part[t].smx;
        if (part[t].hz) ghz = 1;
      }
      if (Ft == 0) {
        /* FitError: the reason histogram over every node */
        for (int r = 0; r < KSIM_NREASONS; ++r) my->hist[r] = 0;
        for (int64_t i = lo; i < hi; ++i)
          for (uint32_t m = mask[i]; m; m &= m - 1) my->hist[__builtin_ctz(m)] += 1;
#pragma omp barrier
#pragma omp single
        {
          if (out_reasons) {
            int32_t* h = &out_reasons[(k - first) * KSIM_NREASONS];
            for (int r = 0; r < KSIM_NREASONS; ++r) {
              h[r] = 0;
              for (int t = 0; t < T_; ++t) h[r] += part[t].hist[r];
            }
          }
          out_node[k - first] = -1;
        }
        continue;  /* the single's barrier ends the pod */
      }
      if (Ft == 1) {
#pragma omp single
        {
          winner = -1;
          for (int64_t i = 0; i < n; ++i)
            if (!mask[i]) { winner = i; break; }
          out_node[k - first] = (int32_t)winner;
          rc = assume_pod(&N, P, pod_ports, pod_scalars, winner);
          if (rc == KSIM_OK && vt && P->vol_class > 0) rc = assume_volumes(&T, P, winner);
          if (rc == KSIM_OK && at && (P->aff_ident > 0 || P->aff_class > 0)) assume_affinity(&T, P, winner);
        }
        continue;
      }
      /* ---- phase 2: reduce + weighted sum over this thread's fit nodes, its (max, count) ---- */
      if (sp >= 0) {
        /* countsByZone over the fit nodes and its maximum (selector_spreading.go:139-143) */
#pragma omp single
        {
          G_zmx = 0;
          for (int z = 0; z < n_zone; ++z) {
            int64_t v = 0;
            for (int t = 0; t < T_; ++t) v += zsum[(size_t)t * (n_zone + 1) + z];
            zall[z] = v;
            if (v > G_zmx) G_zmx = v;
          }
        }
      }
      if (ap >= 0) {
#pragma omp single
        {
          G_azmx = 0;
          for (int z = 0; z < n_adom; ++z) {
            int64_t v = 0;
            for (int t = 0; t < T_; ++t) v += asum[(size_t)t * (n_adom + 1) + z];
            aall[z] = v;
            if (v > G_azmx) G_azmx = v;
          }
        }
      }
      int64_t lM = INT64_MIN, lC = 0;
      for (int64_t i = lo; i < hi; ++i) {
        if (mask[i]) continue;
        uint64_t t = (uint64_t)score[i];
        if (cfg->no_priorities) t = 0;
        if (wt) t += (uint64_t)wt * (uint64_t)normalize(ttv[i], mT, 1);
        if (wa) t += (uint64_t)wa * (uint64_t)normalize(nav[i], mA, 0);
        /* NodePreferAvoidPods (node_prefer_avoid_pods.go:32-68): its weighted map score rides the
           node's NodeAffinity class (ksim_class_tables.na_add) */
        if (ct->na_add)
          t += (uint64_t)ct->na_add[cls * VW(ct) + ct->na_class[cls * ct->n_label_sets + N.label_set[i]]];
        if (ipa && gmx - gmn > 0)  /* fScore = MaxPriority * ((count - min) / (max - min)), :228-236 */
          t += (uint64_t)wi * (uint64_t)(int64_t)(10.0 * ((double)(raw[i] - gmn) / (double)(gmx - gmn)));
        if (sp >= 0) {
          const int64_t c = xs->cnt[at->pair_off[sp] + aff_dom(at, at->pair_key[sp], i)];
          const int32_t z = at->zone_key >= 0 ? aff_dom(at, at->zone_key, i) : -1;
          t += (uint64_t)wsp * (uint64_t)spread_score(c, gsmx, (int)ghz, z, z >= 0 ? zall[z] : 0, G_zmx);
        }
        if (aread) {
          const int64_t c = ap >= 0 ? xs->cnt[at->pair_off[ap] + aff_dom(at, at->pair_key[ap], i)] : 0;
          const int32_t d = aff_dom(at, at->aux_key, i);
          t += (uint64_t)at->aux_weight *
               (uint64_t)aux_score(at->aux_kind, c, d, (ap >= 0 && d >= 0) ? aall[d] : 0, gamx, gatot, (int)gahz, G_azmx);
        }
        score[i] = (int64_t)t;
        if (score[i] > lM) { lM = score[i]; lC = 1; }
        else if (score[i] == lM) lC += 1;
      }
      my->M = lM; my->C = lC;
#pragma omp barrier
      /* ---- selectHost: C = nodes at the max, ix = lastNodeIndex % C from the top; commit ---- */
#pragma omp single
      {
        M = INT64_MIN;
        for (int t = 0; t < T_; ++t)
          if (part[t].C && part[t].M > M) M = part[t].M;
        int64_t C = 0;
        for (int t = 0; t < T_; ++t)
          if (part[t].C && part[t].M == M) C += part[t].C;
        ixv = (int64_t)(counter % (uint64_t)C);
        counter += 1;
        winner = -1;
        int64_t ix = ixv;
        for (int t = T_ - 1; t >= 0 && winner < 0; --t) {  /* descending (score, name rank) */
          if (!part[t].C || part[t].M != M) continue;
          if (ix >= part[t].C) { ix -= part[t].C; continue; }
          const int64_t tlo = n * t / T_, thi = n * (t + 1) / T_;
          for (int64_t i = thi - 1; i >= tlo; --i) {
            if (mask[i] || score[i] != M) continue;
            if (ix == 0) { winner = i; break; }
            --ix;
          }
        }
        out_node[k - first] = (int32_t)winner;
        rc = assume_pod(&N, P, pod_ports, pod_scalars, winner);
        if (rc == KSIM_OK && vt && P->vol_class > 0) rc = assume_volumes(&T, P, winner);
        if (rc == KSIM_OK && at && (P->aff_ident > 0 || P->aff_class > 0)) assume_affinity(&T, P, winner);
      }
    }
  }
  *io_counter = counter;
  free(mask); free(score); free(ttv); free(nav); free(raw); free(zsum); free(zall); free(part); free(asum); free(aall);
  if (rc == KSIM_OK && xs && xs->svc_err) rc = KSIM_E_UNSUPPORTED;
  return rc;
}

/* The resource / selector / port / taint subset (no affinity, spread or volume tables). */
int ksim_ref_run(const ksim_config* cfg, const ksim_node_table* tab, ksim_node_state* st, const ksim_class_tables* ct,
                 const ksim_pod* pods, const uint64_t* pod_ports, const ksim_scalar_req* pod_scalars, int64_t first,
                 int64_t count, int threads, int32_t* out_node, int32_t* out_reasons, uint64_t* io_counter) {
  return ksim_ref_run_ex(cfg, tab, st, ct, NULL, NULL, NULL, pods, pod_ports, pod_scalars, first, count, threads,
                         out_node, out_reasons, io_counter);
}
