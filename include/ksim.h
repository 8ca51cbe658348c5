/*
 * ksim.h — C-ABI of the MI355X-native per-pod scheduling cycle (libksim.so).
 *
 * Drop-in boundary for the vendored kube-scheduler v1.10 hot path that
 * xiaoxubeii/kubernetes-schedule-simulator drives.  The reference interface being
 * replaced is algorithm.ScheduleAlgorithm
 *   (vendor/k8s.io/kubernetes/pkg/scheduler/algorithm/scheduler_interface.go:52-65),
 * installed as scheduler.Config.Algorithm (pkg/scheduler/scheduler.go:109) and built by
 * CreateFromKeys (pkg/scheduler/factory/factory.go:1021-1060) from predicate/priority key
 * sets.  Everything is plain C: fixed-width integers, caller-owned buffers copied in,
 * results written to caller-provided arrays; no pointer is retained past a call (cgo rule).
 * Status: 0 = KSIM_OK, negative = KSIM_E_*, message via ksim_last_error().
 *
 * Node order: every node table is in ascending BYTEWISE name order (Go string <), so a
 * node index is its name rank; selectHost's (score, host) descending sort
 * (core/generic_scheduler.go:183-198, api/types.go:272-277) becomes "largest index first"
 * among the max-score nodes.
 */
#ifndef KSIM_H
#define KSIM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KSIM_ABI_VERSION 7

/* ---- status codes ---- */
#define KSIM_OK 0
#define KSIM_E_INVAL (-1)       /* bad argument / shape */
#define KSIM_E_DEVICE (-2)      /* HIP runtime error */
#define KSIM_E_NOMEM (-3)       /* device allocation failed */
#define KSIM_E_UNSUPPORTED (-4) /* configuration outside the supported key set */
#define KSIM_E_STATE (-5)       /* call order (e.g. schedule before load) */
#define KSIM_E_OVERFLOW (-6)    /* a node's host-port or volume slots overflowed on commit */
#define KSIM_E_NO_NODES (-7)    /* core.ErrNoNodesAvailable (generic_scheduler.go:64,124-125) */

#define KSIM_MAX_SCALAR 8   /* extended / hugepage resource columns */
#define KSIM_MAX_RCLASS 16  /* TaintToleration / NodeAffinity values per pod class (each dimension) in the
                               default value rows; a product above 16 takes the launch form's wide
                               decision, and ksim_class_tables.val_width widens the rows (ABI 7) */
#define KSIM_MAX_WIDE 256   /* reduce classes per pod (TaintToleration x NodeAffinity) */
#define KSIM_NREASONS 32    /* failure-reason histogram slots */
#define KSIM_MAX_RANKS 8    /* devices of one node-sharded cluster */

/* ---- predicate key bits: the FitPredicate keys of predicates.go:129-138 that carry
 *      logic for supported pods.  The volume keys read the tables of ksim_load_volumes and are
 *      true for pods without a volume class.  CheckVolumeBinding needs no bit: it is true for
 *      every pod the host accepts (no PVC, or PVCs bound to PVs without node affinity). ---- */
#define KSIM_P_CHECK_NODE_CONDITION (1u << 0)     /* predicates.go:1534 */
#define KSIM_P_CHECK_NODE_UNSCHEDULABLE (1u << 1) /* CheckNodeUnschedulablePredicate */
#define KSIM_P_GENERAL (1u << 2)                  /* predicates.go:1059 */
#define KSIM_P_HOSTNAME (1u << 3)                 /* predicates.go:853 */
#define KSIM_P_HOST_PORTS (1u << 4)               /* predicates.go:1019 */
#define KSIM_P_NODE_SELECTOR (1u << 5)            /* predicates.go:841 */
#define KSIM_P_RESOURCES (1u << 6)                /* predicates.go:706 */
#define KSIM_P_TAINTS (1u << 7)                   /* predicates.go:1465 */
#define KSIM_P_NOEXEC_TAINTS (1u << 8)            /* PodToleratesNodeNoExecuteTaints */
#define KSIM_P_MEM_PRESSURE (1u << 9)             /* predicates.go:1502 */
#define KSIM_P_DISK_PRESSURE (1u << 10)           /* predicates.go:1524 */
#define KSIM_P_LABEL_PRESENCE (1u << 11)          /* CheckNodeLabelPresence with a labelsPresence
                                                     argument (predicates.go:875-910); the node's
                                                     verdict is the KSIM_N_LABEL_PRESENCE bit */
#define KSIM_P_INTERPOD_AFFINITY (1u << 12)       /* MatchInterPodAffinity (predicates.go:1143-1450),
                                                     over the tables of ksim_load_affinity */
#define KSIM_P_DISK_CONFLICT (1u << 13)           /* NoDiskConflict (predicates.go:220-285) */
#define KSIM_P_MAX_EBS (1u << 14)                 /* MaxEBSVolumeCount (predicates.go:313-456) */
#define KSIM_P_MAX_GCE_PD (1u << 15)              /* MaxGCEPDVolumeCount */
#define KSIM_P_MAX_AZURE_DISK (1u << 16)          /* MaxAzureDiskVolumeCount */
#define KSIM_P_VOLUME_ZONE (1u << 17)             /* NoVolumeZoneConflict (predicates.go:539-633), as the
                                                     per (volume class, label set) verdict zone_ok */
#define KSIM_P_SERVICE_AFFINITY (1u << 18)        /* CheckServiceAffinity with a serviceAffinity argument
                                                     (predicates.go:940-1016), as the per (pod class, label
                                                     set) verdict ksim_class_tables.svc_ok */

/* ---- priority weight slots (0 = not configured).  Priorities that evaluate to the
 *      same value on every node under supported inputs (SelectorSpread /
 *      ServiceSpreading with no selectors, NodePreferAvoidPods for pods without an
 *      RC/RS owner, EqualPriority) do not change placements; their sum goes in
 *      ksim_config.const_score. ---- */
#define KSIM_W_LEAST_REQUESTED 0     /* least_requested.go:36 */
#define KSIM_W_MOST_REQUESTED 1      /* most_requested.go:34 */
#define KSIM_W_BALANCED 2            /* balanced_resource_allocation.go:39 */
#define KSIM_W_TAINT_TOLERATION 3    /* taint_toleration.go:55 + NormalizeReduce(10,true) */
#define KSIM_W_NODE_AFFINITY 4       /* node_affinity.go:34 + NormalizeReduce(10,false) */
#define KSIM_W_INTERPOD_AFFINITY 5   /* interpod_affinity.go:118-240 (0 everywhere without
                                        affinity tables or terms) */
#define KSIM_W_SELECTOR_SPREAD 6     /* SelectorSpreadPriority / ServiceSpreadingPriority
                                        (selector_spreading.go:66-174) for pods whose affinity class
                                        carries a spread pair; other pods score MaxPriority (constant) */
#define KSIM_NW 7

/* ---- node condition / dynamic flags (ksim_node_table.flags) ---- */
#define KSIM_N_NOT_READY (1u << 0)      /* Ready condition present, status != True */
#define KSIM_N_OUT_OF_DISK (1u << 1)    /* OutOfDisk present, status != False */
#define KSIM_N_NET_UNAVAIL (1u << 2)    /* NetworkUnavailable present, != False */
#define KSIM_N_UNSCHEDULABLE (1u << 3)  /* spec.unschedulable */
#define KSIM_N_MEM_PRESSURE (1u << 4)   /* MemoryPressure == True */
#define KSIM_N_DISK_PRESSURE (1u << 5)  /* DiskPressure == True */
#define KSIM_N_LABEL_PRESENCE (1u << 6) /* the node fails the policy's CheckNodeLabelPresence */
#define KSIM_N_GPU_OVER (1u << 8)       /* alloc.gpu < requested.gpu  (maintained by the library) */
#define KSIM_N_EPH_OVER (1u << 9)       /* alloc.eph < requested.eph  (maintained by the library) */

/* ---- pod flags (ksim_pod.flags) ---- */
#define KSIM_POD_ANY_REQUEST (1u << 0)  /* PodFitsResources does the resource checks (:731-736) */
#define KSIM_POD_BEST_EFFORT (1u << 1)  /* qos.go:39 BestEffort */
#define KSIM_POD_NEED_SELECTOR (1u << 2)/* nodeSelector/required affinity not matching every label set */
#define KSIM_POD_NEED_TAINTS (1u << 3)  /* some taint set is not tolerated */
#define KSIM_POD_NEED_SVC_AFFINITY (1u << 4) /* CheckServiceAffinity fails on some label set (launch kernels) */

/* ---- failure reasons: bit r of a node's reason mask / slot r of a histogram ---- */
#define KSIM_R_NOT_READY 0
#define KSIM_R_OUT_OF_DISK 1
#define KSIM_R_NET_UNAVAIL 2
#define KSIM_R_UNSCHEDULABLE 3
#define KSIM_R_INSUFFICIENT_PODS 4
#define KSIM_R_INSUFFICIENT_CPU 5
#define KSIM_R_INSUFFICIENT_MEMORY 6
#define KSIM_R_INSUFFICIENT_GPU 7
#define KSIM_R_INSUFFICIENT_EPHEMERAL 8
#define KSIM_R_HOSTNAME 9
#define KSIM_R_HOST_PORTS 10
#define KSIM_R_NODE_SELECTOR 11
#define KSIM_R_TAINTS 12
#define KSIM_R_MEM_PRESSURE 13
#define KSIM_R_DISK_PRESSURE 14
#define KSIM_R_LABEL_PRESENCE 15
#define KSIM_R_INSUFFICIENT_SCALAR0 16 /* +column, up to KSIM_MAX_SCALAR */
/* MatchInterPodAffinity fails with two reasons (predicates.go:1149-1160): the generic one
 * plus the rule that failed (algorithm/predicates/error.go:40-47) */
#define KSIM_R_POD_AFFINITY 24            /* node(s) didn't match pod affinity/anti-affinity */
#define KSIM_R_EXISTING_ANTI_AFFINITY 25  /* node(s) didn't satisfy existing pods anti-affinity rules */
#define KSIM_R_AFFINITY_RULES 26          /* node(s) didn't match pod affinity rules */
#define KSIM_R_ANTI_AFFINITY_RULES 27     /* node(s) didn't match pod anti-affinity rules */
#define KSIM_R_DISK_CONFLICT 28           /* node(s) had no available disk (ErrDiskConflict) */
#define KSIM_R_MAX_VOLUME_COUNT 29        /* node(s) exceed max volume count (ErrMaxVolumeCountExceeded) */
#define KSIM_R_VOLUME_ZONE 30             /* node(s) had no available volume zone (ErrVolumeZoneConflict) */
#define KSIM_R_SERVICE_AFFINITY 31        /* node(s) didn't match service affinity (ErrServiceAffinityViolated) */

/* ---- execution modes ---- */
#define KSIM_MODE_AUTO 0        /* library picks (persistent when it fits) */
#define KSIM_MODE_LAUNCH 1      /* one scan launch per pod, replayed from a hipGraph */
#define KSIM_MODE_PERSISTENT 2  /* one persistent launch walks the whole pod queue */
/* Incremental per-pod-class selection trees: resource-only pods under
 * map-only policies are decided from a tree that each commit updates along one leaf-to-root
 * path, O(classes x log N) per pod instead of the O(N) scan; same placements.  Runs of other
 * pods in the range, and tables/class sets beyond the tree's limits, take the AUTO path. */
#define KSIM_MODE_TREE 3

typedef struct {
  int32_t device;                 /* HIP device ordinal */
  int32_t mode;                   /* KSIM_MODE_* */
  uint32_t predicates;            /* KSIM_P_* bits of the configured key set */
  int64_t weights[KSIM_NW];       /* PriorityConfig.Weight per slot (Go int) */
  int32_t no_priorities;          /* 1: empty prioritizer list -> EqualPriorityMap */
  int32_t collect_reasons;        /* 1: fill failure histograms for unschedulable pods */
  int64_t const_score;            /* sum of constant-valued priorities (reporting only) */
  uint64_t last_node_index;       /* initial genericScheduler.lastNodeIndex */
} ksim_config;

/* Node table in name-rank order.  Column arrays have n_nodes entries; scalar columns are
 * [n_scalar][n_nodes]; ports are slot-major [port_slots][n_nodes] with 0 = empty. */
typedef struct {
  int64_t n_nodes;
  int32_t n_scalar;
  int32_t port_slots;
  /* static (NodeInfo.SetNode, node_info.go:429-448) */
  const int64_t* alloc_cpu;   /* milli */
  const int64_t* alloc_mem;
  const int64_t* alloc_gpu;
  const int64_t* alloc_eph;
  const int32_t* allowed_pods;
  const uint32_t* flags;      /* KSIM_N_* condition bits (the library derives _OVER bits) */
  const int32_t* label_set;   /* interned label-set id */
  const int32_t* taint_set;   /* interned taint-set id */
  const int64_t* alloc_scalar;
  /* dynamic (NodeInfo.AddPod, node_info.go:318-341) — state from already running pods */
  const int64_t* req_cpu;
  const int64_t* req_mem;
  const int64_t* req_gpu;
  const int64_t* req_eph;
  const int64_t* nz_cpu;
  const int64_t* nz_mem;
  const int32_t* pod_count;
  const int64_t* req_scalar;
  const uint64_t* ports;      /* KSIM_PORT_KEY(ip_id, proto_id, port) */
  const int32_t* port_count;
} ksim_node_table;

#define KSIM_PORT_KEY(ip, proto, port) \
  ((((uint64_t)(ip)) << 40) | (((uint64_t)(proto)) << 32) | (uint64_t)(uint32_t)(port))

/* Per pod-class tables (pods with identical specs share a class).  Bit tables are
 * [n_classes][words] with words = ceil(n_sets/32); byte tables are [n_classes][n_sets]. */
typedef struct {
  int32_t n_classes;
  int32_t n_label_sets;
  int32_t n_taint_sets;
  const uint32_t* sel_ok;      /* podMatchesNodeLabels per label set (predicates.go:795) */
  const uint32_t* taint_ok;    /* NoSchedule+NoExecute tolerated per taint set (:1465) */
  const uint32_t* noexec_ok;   /* NoExecute tolerated per taint set */
  const uint8_t* tt_class;     /* reduce class of each taint set (intolerable PreferNoSchedule count) */
  const uint8_t* na_class;     /* reduce class of each label set (preferred node-affinity weight) */
  const int32_t* n_tt;         /* [n_classes] number of TaintToleration classes K1 */
  const int32_t* n_na;         /* [n_classes] number of NodeAffinity classes K2 (each <= the value row
                                  width, K1*K2 <= KSIM_MAX_WIDE; above 16 the launch form decides) */
  const int64_t* tt_val;       /* [n_classes][width] map value of each class (width: val_width) */
  const int64_t* na_val;       /* [n_classes][width] */
  /* Optional (NULL = none): a weighted constant added to the total of every node of NodeAffinity
   * class b, [n_classes][KSIM_MAX_RCLASS] — NodePreferAvoidPodsPriority's map score x weight
   * (node_prefer_avoid_pods.go:32-68), which is a function of (pod class, label set) like the
   * NodeAffinity value.  When set, the NodeAffinity class dimension is used whatever
   * NodeAffinityPriority's weight (n_na then counts (preferred weight, avoid score) pairs). */
  const int64_t* na_add;
  /* Optional (NULL = every node passes): CheckServiceAffinity's verdict per label set,
   * [n_classes][words] like sel_ok — the pod's nodeSelector values of the predicate's labels must
   * be the node's (FindLabelsInSet, CreateSelectorFromLabels; no service selects the pod). */
  const uint32_t* svc_ok;
  /* The row width of tt_val / na_val / na_add (0 = KSIM_MAX_RCLASS; at most KSIM_MAX_WIDE): a pod
   * class with more than 16 TaintToleration or NodeAffinity values (NormalizeReduce has no such
   * limit, reduce.go:29-64) needs rows as wide as its larger dimension. */
  int32_t val_width;
  int32_t reserved0;
} ksim_class_tables;

/* Pod descriptor, 128 bytes.  The three request vectors follow the reference exactly:
 * req_* = GetResourceRequest (predicates.go:659-697, init containers max'd in),
 * add_* = calculateResource (node_info.go:400-412, containers only),
 * nz_*  = non-zero requests (priorities/util/non_zero.go:38-53). */
typedef struct {
  int64_t req_cpu, req_mem, req_gpu, req_eph;
  int64_t add_cpu, add_mem, add_gpu, add_eph;
  int64_t nz_cpu, nz_mem;
  int32_t cls;         /* pod class */
  int32_t host;        /* spec.nodeName: -1 none, >=0 node index, -2 names no node */
  uint32_t flags;      /* KSIM_POD_* */
  int32_t port_off;    /* into the pod-port array */
  int32_t port_cnt;
  int32_t scalar_off;  /* into the scalar-request array */
  int32_t scalar_cnt;
  int32_t aff_ident;   /* 1 + identity in the affinity tables (ksim_load_affinity); 0: none */
  int32_t aff_class;   /* 1 + affinity class (own and carried terms); 0: none */
  int32_t vol_class;   /* 1 + volume class in the tables of ksim_load_volumes; 0: no relevant volume */
  int32_t reserved[2]; /* library-owned scratch (callers pass anything; never read back) */
} ksim_pod;

typedef struct {
  int32_t col;     /* scalar column */
  int32_t pad;
  int64_t req;     /* predicate request */
  int64_t add;     /* commit delta */
} ksim_scalar_req;

typedef struct {
  int64_t pods;            /* pods processed by the call */
  int64_t scheduled;       /* pods bound */
  int64_t node_evals;      /* sum over pods of nodes scanned */
  double device_ms;        /* HIP-event time of the call's device work */
  double kernel_ms;        /* HIP-event time of the dominant (scan) kernel(s) */
  int64_t kernel_launches; /* launches of the dominant kernel */
  int32_t mode;            /* mode actually used */
  int32_t blocks;          /* grid size of the dominant kernel */
} ksim_stats;

/* Dynamic node columns read back by ksim_read_nodes (caller-provided arrays or NULL). */
typedef struct {
  int64_t* req_cpu;
  int64_t* req_mem;
  int64_t* req_gpu;
  int64_t* req_eph;
  int64_t* nz_cpu;
  int64_t* nz_mem;
  int32_t* pod_count;
  int64_t* req_scalar;   /* [n_scalar][n_nodes] */
  uint64_t* ports;       /* [port_slots][n_nodes] */
  int32_t* port_count;
} ksim_node_state;

typedef struct ksim_handle ksim_handle;

int ksim_abi_version(void);
const char* ksim_last_error(const ksim_handle* h);   /* h may be NULL (global error) */

/* Create a handle bound to cfg->device; replaces algorithm.ScheduleAlgorithm construction
 * (core/generic_scheduler.go:1088 NewGenericScheduler). */
int ksim_create(const ksim_config* cfg, ksim_handle** out);
void ksim_destroy(ksim_handle* h);

/* Snapshot ingest: the node cache (schedulercache UpdateNodeNameToInfoMap, cache.go:83). */
int ksim_load_nodes(ksim_handle* h, const ksim_node_table* nodes);
/* May be called again with a superset (new pod classes, label sets, taint sets). */
int ksim_load_classes(ksim_handle* h, const ksim_class_tables* classes);
/* Pod queue in scheduling order (the simulator's LIFO PodQueue.Pop order, store.go:223). */
int ksim_load_pods(ksim_handle* h, const ksim_pod* pods, int64_t n_pods, const uint64_t* ports,
                   int64_t n_ports, const ksim_scalar_req* scalars, int64_t n_scalars);

/* Schedule pods [first, first+count) of the loaded queue in order, committing each
 * placement (Scheduler.assume → NodeInfo.AddPod) before the next pod.  out_node[i] is the
 * node index or -1 (FitError).  out_reasons (optional, [count][KSIM_NREASONS]) receives the
 * FitError reason histogram of unschedulable pods (generic_scheduler.go:72-90). */
int ksim_schedule(ksim_handle* h, int64_t first, int64_t count, int32_t* out_node,
                  int32_t* out_reasons, ksim_stats* stats);

/* Evaluate one loaded pod against the current node state without committing and without
 * touching lastNodeIndex: per-node fit, reason mask (first failing predicate in
 * predicatesOrdering), map score and reduce class. */
int ksim_evaluate(ksim_handle* h, int64_t pod, uint8_t* out_fit, uint32_t* out_reasons,
                  int64_t* out_score, uint8_t* out_rclass);

/* Scenario sweep — the capacity-planning what-if (BASELINE configs[4]): n_scen
 * independent copies of the current node state each schedule pods [first, first+count) in order
 * under their own map-priority weights (weights[s*KSIM_NW + KSIM_W_LEAST_REQUESTED /
 * _MOST_REQUESTED / _BALANCED]; the reduce slots must be 0), starting from the current
 * lastNodeIndex, with the configured predicates.  Replaces running the simulator once per
 * policy (pkg/scheduler/simulator.go:286 New, :187 Run).  Every pod must be resource-only;
 * the handle's own state is left unchanged.  out_node: [n_scen][count] node index or -1;
 * out_counters (optional): [n_scen] final lastNodeIndex. */
int ksim_sweep(ksim_handle* h, const int64_t* weights, int32_t n_scen, int64_t first, int64_t count,
               int32_t* out_node, uint64_t* out_counters, ksim_stats* stats);

/* ---- Node-sharded scheduling of one cluster across devices ----
 * Rank r of `world` (one handle per device, one process or thread each) loads the contiguous
 * name-rank shard [node_base, node_base + n_r) of the node table and the whole pod queue.
 * Every rank then calls ksim_schedule with the same (first, count) sequence; per pod the
 * ranks combine their (fit count, max score, count at max) through device-initiated writes
 * into each other's exchange buffers (xGMI), reach the same findNodesThatFit / selectHost
 * decision (core/generic_scheduler.go:112-198) and the owning rank commits.  out_node on
 * rank r: the global node index if rank r holds it, -1 (FitError), -2 (another rank's node).
 * Only resource-only pods are supported in this mode (KSIM_E_UNSUPPORTED otherwise). */
#define KSIM_IPC_HANDLE_BYTES 64
int ksim_shard_setup(ksim_handle* h, int32_t rank, int32_t world, int64_t node_base);
/* IPC handle of this rank's exchange buffer, to be passed to every other rank. */
int ksim_shard_export(ksim_handle* h, uint8_t* out_handle);
/* Map rank `peer`'s exchange buffer (another process). */
int ksim_shard_connect(ksim_handle* h, int32_t peer, const uint8_t* peer_handle);
/* Same, for a rank driven from this process (its handle). */
int ksim_shard_connect_local(ksim_handle* h, int32_t peer, ksim_handle* peer_h);

/* Commit one loaded pod to a node (Scheduler.assume / cache.AssumePod). */
int ksim_assume(ksim_handle* h, int64_t pod, int64_t node);

/* ==== Per-pod drop-in and scheduler-cache sync ===========================================
 * The reference calls ScheduleAlgorithm.Schedule(pod, nodeLister) once per pod
 * (algorithm/scheduler_interface.go:52-65) from Scheduler.schedule (scheduler.go:188-204), then
 * Scheduler.assume (scheduler.go:366) → schedulerCache.AssumePod (schedulercache/cache.go:125).
 * Informer events keep the cache in sync: addPodToCache / deletePodFromCache
 * (factory/factory.go:596,695) → cache.AddPod / RemovePod (cache.go:230,292), addNodeToCache /
 * updateNodeInCache / deleteNodeFromCache (factory.go:740,755,841) → cache.AddNode / UpdateNode /
 * RemoveNode (cache.go:354,366,378).  These entry points are that surface on the device-resident
 * table: a pod is passed as a descriptor (its port_off / scalar_off index the arrays passed with
 * it), nodes are addressed by name rank (the caller keeps the bytewise-sorted name list; an
 * insert at rank r moves ranks >= r up by one).  None of them needs a loaded pod queue. */

/* Result of one Schedule call. */
typedef struct {
  int32_t node;                    /* selected node (name rank), -1: FitError */
  int32_t fit_nodes;               /* len(filtered) of findNodesThatFit (generic_scheduler.go:136) */
  uint64_t last_node_index;        /* genericScheduler.lastNodeIndex after the call */
  int32_t reasons[KSIM_NREASONS];  /* FitError.FailedPredicates histogram when node == -1 */
} ksim_result;

#define KSIM_SCHEDULE_ONLY 0    /* genericScheduler.Schedule: decide, leave the cache unchanged */
#define KSIM_SCHEDULE_ASSUME 1  /* Schedule + Scheduler.assume (AssumePod on the chosen node) */

/* One pod through findNodesThatFit → PrioritizeNodes → selectHost (one scan launch, no
 * queue), optionally assumed.  ports [n_ports] / scalars [n_scalars] are the pod's host-port
 * keys and scalar requests (pod->port_off / scalar_off index them).  Returns KSIM_OK with
 * out->node == -1 for a FitError, KSIM_E_NO_NODES when the table is empty. */
int ksim_schedule_one(ksim_handle* h, const ksim_pod* pod, const uint64_t* ports, int32_t n_ports,
                      const ksim_scalar_req* scalars, int32_t n_scalars, int32_t assume, ksim_result* out);

/* NodeInfo.AddPod / RemovePod on node `node` (name rank) for a pod descriptor: cache.AddPod of a
 * pod bound elsewhere, AssumePod after a KSIM_SCHEDULE_ONLY decision, cache.RemovePod
 * (node_info.go:318-390).  The caller's cache mirror owns pod identity (the "no corresponding
 * pod" error of RemovePod); the library applies the resource / port delta. */
int ksim_pod_add(ksim_handle* h, int64_t node, const ksim_pod* pod, const uint64_t* ports, int32_t n_ports,
                 const ksim_scalar_req* scalars, int32_t n_scalars);
int ksim_pod_remove(ksim_handle* h, int64_t node, const ksim_pod* pod, const uint64_t* ports, int32_t n_ports,
                    const ksim_scalar_req* scalars, int32_t n_scalars);

/* One node's columns (the row of ksim_node_table): static ones as NodeInfo.SetNode derives them
 * (node_info.go:429-448), dynamic ones for pods already on the node. */
typedef struct {
  int64_t alloc_cpu, alloc_mem, alloc_gpu, alloc_eph;
  int32_t allowed_pods;
  uint32_t flags;               /* KSIM_N_* condition bits */
  int32_t label_set, taint_set; /* ids in the loaded class tables */
  int64_t req_cpu, req_mem, req_gpu, req_eph, nz_cpu, nz_mem;
  int32_t pod_count, port_count;
  const int64_t* alloc_scalar;  /* [n_scalar] or NULL */
  const int64_t* req_scalar;    /* [n_scalar] or NULL */
  const uint64_t* ports;        /* [port_count] KSIM_PORT_KEY or NULL */
} ksim_node_row;

/* cache.AddNode of a node whose bytewise name rank among the listed nodes is `index`
 * (0..n): rows index.. move up one, queued pods' spec.nodeName ranks follow. */
int ksim_node_add(ksim_handle* h, int64_t index, const ksim_node_row* row);
/* cache.UpdateNode → SetNode: the static columns of row `index` (dynamic ones are kept). */
int ksim_node_update(ksim_handle* h, int64_t index, const ksim_node_row* row);
/* cache.RemoveNode: the node leaves the listed set (nodeLister.List no longer returns it). */
int ksim_node_remove(ksim_handle* h, int64_t index);
int ksim_node_count(ksim_handle* h, int64_t* out);

/* Append pods to the loaded queue (first call may also be ksim_load_pods): offsets in the
 * new descriptors index the arrays passed with them.  New pod classes need the class tables
 * reloaded first (ksim_load_classes may be called again with a superset). */
int ksim_append_pods(ksim_handle* h, const ksim_pod* pods, int64_t n_pods, const uint64_t* ports, int64_t n_ports,
                     const ksim_scalar_req* scalars, int64_t n_scalars);

/* ==== Inter-pod affinity (MatchInterPodAffinity, InterPodAffinityPriority) ==================
 * Reference: algorithm/predicates/predicates.go:1143-1450 (+ metadata.go:102-123),
 * algorithm/priorities/interpod_affinity.go:118-240, priorities/util/topologies.go:28-71.
 * The host interns every string test (ksim/affinity.py):
 *  - topology keys k: dom[k][n] = node n's domain under key k (its value of label k, interned),
 *    -1 when the node lacks the label.  Keys 0 and 1 are pseudo keys: 0 puts every node in
 *    domain 0 ("a matching pod exists anywhere"), 1 puts node n in domain n (hostname terms,
 *    which look only at the node's own pods, predicates.go:1176-1179);
 *  - selectors s: a term's (namespaces, label selector) as its defining pod resolves them;
 *  - identities (namespace, labels) of pods: bit s of ident_sel[i][.] (sel_words 64-bit words per
 *    identity) = the identity matches selector s; bit e of ident_anti / ident_prio[i][.]
 *    (carry_words words) = it matches carried term e (required anti-affinity / priority terms);
 *  - counted pairs (s, k): per domain of k, the number of placed pods matching s;
 *  - carried terms e: terms of placed pods acting on later pods: per domain of the term's
 *    key, the number (required anti-affinity) or summed signed weight (priority terms) of placed
 *    pods carrying it;
 *  - affinity classes: a pod's own terms (required affinity, then required anti-affinity, then
 *    preferred) and the carried amounts it brings; ac[a] = {req_off, req_cnt, pref_off, pref_cnt,
 *    carry_off, carry_cnt}; and its SelectorSpread pair (spread_pair[a]).
 * ksim_pod.aff_ident / aff_class hold 1 + the id (0 = none, so zero-initialised descriptors
 * take no part).  A pod with either set is scheduled by the launch-mode kernels, which apply
 * its counts on commit; the node events (ksim_node_add / update / remove) make the tables stale
 * until they are loaded again. */
#define KSIM_AFF_REQ_AFFINITY 0  /* required pod affinity term */
#define KSIM_AFF_REQ_ANTI 1      /* required pod anti-affinity term */
#define KSIM_AFF_PREFERRED 2     /* preferred term (affinity: +weight, anti-affinity: -weight) */
#define KSIM_AFF_CARRY_ANTI 0    /* carried: an existing pod's required anti-affinity */
#define KSIM_AFF_CARRY_PRIO 1    /* carried: symmetric priority term (hard weight or +-weight) */
#define KSIM_AFF_MAX_SEL 65536
#define KSIM_AFF_MAX_CARRY 65536

typedef struct {
  int32_t kind;        /* KSIM_AFF_REQ_AFFINITY / _REQ_ANTI / _PREFERRED */
  int32_t pair;        /* counted pair read at the node's domain */
  int32_t gate_key;    /* required terms: key the node must carry */
  int32_t exist_pair;  /* required affinity: a count > 0 at the node's domain = a matching pod exists */
  int32_t self_ok;     /* required affinity: the pod matches its own term */
  int32_t pad;
  int64_t weight;      /* preferred: signed weight */
} ksim_aff_term;

typedef struct {
  int32_t term;        /* carried term */
  int32_t pad;
  int64_t amount;      /* 1 (required anti-affinity) or the signed priority weight */
} ksim_aff_carry;

#define KSIM_SVC_LABELS 8
typedef struct {
  int32_t pair_all;                      /* (s_v, key 0): the matching cached pods */
  int32_t pad;
  int32_t pair_present[KSIM_SVC_LABELS]; /* (s_v, presence key of label l) */
  int32_t pair_value[KSIM_SVC_LABELS];   /* (s_v, key of label l) */
} ksim_svc_ident;

typedef struct {
  int32_t n_keys, n_sel, n_ident, n_pair, n_carry, n_aclass;
  int32_t n_terms, n_carries;
  int64_t n_nodes;                 /* must equal the loaded node table's */
  int64_t cnt_len, carried_len;
  int32_t hard_weight;             /* hardPodAffinitySymmetricWeight the carried amounts use */
  int32_t sel_words;               /* ceil(n_sel / 64) */
  int32_t carry_words;             /* ceil(n_carry / 64) */
  int32_t zone_key;                /* key whose domains are the nodes' zones (utilnode.GetZoneKey), the
                                      SelectorSpread reduce's countsByZone; -1: none */
  const int32_t* dom;              /* [n_keys][n_nodes] */
  const int32_t* n_dom;            /* [n_keys] */
  const uint64_t* ident_sel;       /* [n_ident][sel_words] */
  const uint64_t* ident_anti;      /* [n_ident][carry_words] */
  const uint64_t* ident_prio;      /* [n_ident][carry_words] */
  const int32_t* pair_sel;         /* [n_pair] */
  const int32_t* pair_key;         /* [n_pair] */
  const int64_t* pair_off;         /* [n_pair] into cnt (n_dom[pair_key] entries) */
  const int32_t* carry_key;        /* [n_carry] */
  const int32_t* carry_kind;       /* [n_carry] KSIM_AFF_CARRY_* */
  const int64_t* carry_off;        /* [n_carry] into carried */
  const int32_t* ac;               /* [n_aclass][6] */
  const ksim_aff_term* terms;      /* [n_terms] */
  const ksim_aff_carry* carries;   /* [n_carries] */
  const int32_t* cnt;              /* [cnt_len] counts of the pods already placed */
  const int64_t* carried;          /* [carried_len] */
  /* SelectorSpread (selector_spreading.go:66-174): per affinity class the counted pair (s, key 1) of
   * the class's spread selector — s matches the identities, in the pod's namespace and not being
   * deleted, that any of the pod's service / RC / RS / StatefulSet selectors selects — or -1;
   * NULL: no class spreads. */
  const int32_t* spread_pair;      /* [n_aclass] */
  /* One auxiliary counted priority next to the slots of ksim_config.weights (a Policy's second
   * spreading priority), NULL aux_pair: none.  aux_pair[a]: class a's counted pair (s, key 1) or -1;
   * aux_key groups the fit nodes' counts by its domains; aux_weight: the priority's weight.
   *  - KSIM_AUX_SPREAD: SelectorSpread's reduce (selector_spreading.go:121-174) over the pair, zones
   *    from aux_key (ServiceSpreadingPriority configured next to SelectorSpreadPriority: its
   *    services-only selectors);
   *  - KSIM_AUX_SERVICE_ANTI: ServiceAntiAffinity (selector_spreading.go:180-275, a Policy priority
   *    with a serviceAntiAffinity argument): the pair counts the pods of the pod's single selecting
   *    service; a fit node without the aux_key label scores 0, one with value v
   *    MaxPriority x (total - count(v)) / total over the fit nodes (MaxPriority when total = 0, and
   *    for a class without a pair).  Read by the launch-form kernels, the general persistent
   *    kernel (<= 64 aux_key domains) and every per-pod form; with it loaded every pod of a batch
   *    goes to those (a serviceAntiAffinity priority scores pods no service selects too). */
  const int32_t* aux_pair;         /* [n_aclass] or NULL */
  int32_t aux_key;                 /* -1 with aux_pair NULL */
  int32_t aux_kind;                /* KSIM_AUX_* */
  int64_t aux_weight;
  /* CheckServiceAffinity for pods a service selects whose nodeSelector lacks some of the
   * predicate's labels (predicates.go:920-1016): the missing labels take the values of the node
   * of the first cached pod with the pod's labels in its namespace (serviceAffinityMetadataProducer,
   * a pod-lister order), so the library checks that every such pod's node agrees on them and
   * refuses the run (KSIM_E_UNSUPPORTED, the order would decide) when they do not.  Per service-
   * affinity identity v (namespace + labels of such pods): selector s_v (namespace, the labels as a
   * set selector) with counted pairs (s_v, key 0) — the matching cached pods — and per predicate
   * label l (s_v, presence key of l: domain 0 on nodes carrying l) and (s_v, key of l).  NULL
   * svc_ident: none.  Read by the launch-form kernels, the general persistent kernel (<= 256
   * counted pairs) and every per-pod form (the resident one without tentative commits). */
  int32_t n_svc;                   /* service-affinity identities */
  int32_t n_svc_labels;            /* the predicate's labels (<= KSIM_SVC_LABELS) */
  const ksim_svc_ident* svc_ident; /* [n_svc] */
  const int32_t* svc_class;        /* [n_aclass]: the class's identity v, or -1 */
  const uint32_t* svc_miss;        /* [n_aclass]: bit l = the class's nodeSelector lacks label l */
  const uint32_t* svc_conflict;    /* [n_svc]: bit l = the cached pods of v disagree on label l */
  const int32_t* svc_of_off;       /* [n_ident + 1] offsets into svc_of */
  const int32_t* svc_of;           /* the identities v whose selector an affinity identity matches */
} ksim_affinity_tables;
#define KSIM_AUX_SPREAD 0
#define KSIM_AUX_SERVICE_ANTI 1

/* Load (or replace) the affinity tables; the counts describe the pods already placed. */
int ksim_load_affinity(ksim_handle* h, const ksim_affinity_tables* t);

/* ==== Volumes (NoDiskConflict, MaxEBS / GCEPD / AzureDiskVolumeCount, NoVolumeZoneConflict) ====
 * Reference: algorithm/predicates/predicates.go:220-285 (isVolumeConflict, NoDiskConflict),
 * :313-507 (MaxPDVolumeCountChecker, the EBS / GCE PD / Azure Disk filters), :539-633
 * (VolumeZoneChecker).  The host interns every volume identity into a key (ksim/volumes.py):
 *  - GCE PD by PDName, AWS EBS by VolumeID, Azure Disk by DiskName, ISCSI by IQN, RBD once per
 *    Ceph monitor as (monitor, pool, image) — isVolumeConflict's haveOverlap becomes "some key
 *    of the volume is mounted" — and a PVC the PV / PVC listers cannot resolve as
 *    "<namespace>/<claim>" (counted by every MaxPD filter, :376-403).  A PVC bound to a known PV
 *    is the PV's GCE PD / EBS / Azure Disk key, or nothing;
 *  - key_filter[k]: the MaxPD filters (KSIM_VOL_EBS / _GCE_PD / _AZURE_DISK) that count key k;
 *  - volume classes (pods with identical volume lists): refs[vc[c][0] .. + vc[c][1]] with the
 *    flags below, vc_filter[c] = the filters with a relevant volume in the pod (MaxPD's
 *    len(newVolumes) == 0 quick return, :427-430);
 *  - node state: per node the mounted keys with three mount counts — read-write and read-only
 *    mounts by inline volumes (what isVolumeConflict sees) and mounts through a PVC (seen only by
 *    the MaxPD counts) — slot-major [vol_slots][n_nodes] KSIM_VOL_SLOT words (0 = empty) and a
 *    used-slot count; each commit adds the pod's refs, ksim_pod_remove subtracts them (a slot whose
 *    counts reach 0 goes; a count at its field's maximum is a KSIM_E_OVERFLOW);
 *  - zone_ok (optional): [n_vclass][zone_words] bit per label set, NoVolumeZoneConflict's verdict
 *    (a function of the node's zone / region labels and the class's PV labels).
 * A pod with vol_class set is scheduled by the launch-mode kernels; node events (ksim_node_add /
 * update / remove) make the tables stale until they are loaded again. */
#define KSIM_VOL_EBS 1u
#define KSIM_VOL_GCE_PD 2u
#define KSIM_VOL_AZURE_DISK 4u
#define KSIM_VOL_CONFLICT_ANY (1u << 0) /* NoDiskConflict: any mount of the key conflicts (EBS; read-write
                                           GCE PD / ISCSI / RBD) */
#define KSIM_VOL_CONFLICT_RW (1u << 1)  /* NoDiskConflict: read-write mounts conflict (read-only GCE PD /
                                           ISCSI / RBD) */
#define KSIM_VOL_READ_ONLY (1u << 2)    /* the mount counts as read-only */
#define KSIM_VOL_NEW (1u << 3)          /* first ref of the key in the class: one of MaxPD's newVolumes */
#define KSIM_VOL_VIA_PVC (1u << 4)      /* mounted through a PVC: counted by MaxPD, invisible to NoDiskConflict */
/* slot word: key | pvc mounts (10 bits) | read-only inline mounts (11) | read-write inline mounts (11) */
#define KSIM_VOL_SLOT(key, rw, ro, pvc)                                                                   \
  ((((uint64_t)(uint32_t)(key)) << 32) | (((uint64_t)(pvc) & 0x3FFu) << 22) | (((uint64_t)(ro) & 0x7FFu) << 11) | \
   ((uint64_t)(rw) & 0x7FFu))

typedef struct {
  int32_t key;
  uint32_t flags; /* KSIM_VOL_CONFLICT_* | KSIM_VOL_READ_ONLY | KSIM_VOL_NEW | KSIM_VOL_VIA_PVC */
} ksim_vol_ref;

typedef struct {
  int32_t n_keys, n_vclass, n_refs, vol_slots;
  int64_t n_nodes;             /* must equal the loaded node table's */
  int32_t max_vols[3];         /* MaxPD limits: EBS, GCE PD, Azure Disk (getMaxVols, :347-359) */
  int32_t zone_words;          /* ceil(n_label_sets / 32) of the loaded class tables, or 0 without zone_ok */
  const uint32_t* key_filter;  /* [n_keys] */
  const int32_t* vc;           /* [n_vclass][2] (offset, count) into refs */
  const uint32_t* vc_filter;   /* [n_vclass] */
  const ksim_vol_ref* refs;    /* [n_refs] */
  const uint32_t* zone_ok;     /* [n_vclass][zone_words] or NULL (every node passes) */
  const uint64_t* slots;       /* [vol_slots][n_nodes] mounts of the pods already placed */
  const int32_t* slot_count;   /* [n_nodes] */
} ksim_volume_tables;

/* Load (or replace) the volume tables; the slots describe the pods already placed. */
int ksim_load_volumes(ksim_handle* h, const ksim_volume_tables* t);
/* Grow the loaded volume tables for a pod that brings new volume keys / classes (the per-pod
 * path; predicates.go:287-507 read them): key_filter, vc, vc_filter, refs and zone_ok are replaced
 * (each at least as large as before, existing entries unchanged), vol_slots may grow, and slots /
 * slot_count are ignored (may be NULL) — the device keeps every node's mounts, so the cost is the
 * small tables, not the cached pods.  KSIM_E_STATE after a node event (reload with
 * ksim_load_volumes).  Replaces the rebuild the reference never needs: its NodeInfo holds the
 * pods and predicateMetadata grows with them (schedulercache/cache.go:200-318). */
int ksim_grow_volumes(ksim_handle* h, const ksim_volume_tables* t);
/* Read back the volume slots ([vol_slots][n_nodes]) and counts ([n_nodes]); either may be NULL. */
int ksim_read_volumes(ksim_handle* h, uint64_t* slots, int32_t* slot_count);

int ksim_read_nodes(ksim_handle* h, ksim_node_state* out);
int ksim_get_counter(ksim_handle* h, uint64_t* out);
int ksim_set_counter(ksim_handle* h, uint64_t value);

/* Device self-test of the wave64 DPP reduction/scan helpers the kernels use (diagnostic):
 * returns the number of mismatching lanes against plain lane loops (0 = pass, <0 = error). */
int ksim_selftest(void);

#ifdef __cplusplus
}
#endif
#endif /* KSIM_H */
