/* ksim_k8s.h — the Kubernetes-field front end of libksim: v1.Node / v1.Pod / PV / PVC fields in,
 * device tables out.  Everything the scheduler decides by comparing strings — label selectors
 * (apimachinery labels/selector.go:193-215, 837-853), node selectors and node affinity
 * (algorithm/predicates/predicates.go:780-838), tolerations (core/v1/toleration.go:37-56, predicates
 * .go:1465-1494), inter-pod affinity terms with their namespaces and topology keys
 * (predicates.go:1143-1450, priorities/interpod_affinity.go:118-240, priorities/util/topologies.go),
 * SelectorSpread selectors and zones (priorities/selector_spreading.go:66-174), volume identities
 * and their listers (predicates.go:220-633), NodePreferAvoidPods signatures
 * (priorities/node_prefer_avoid_pods.go:32-68) — is interned and evaluated here, in C++, into the
 * tables of include/ksim.h.  A cgo adapter flattens the Go objects into these structs and never
 * re-implements a scheduling rule.
 *
 * Conventions: strings are NUL-terminated UTF-8 and may be NULL where "absent" and "" mean the same
 * to the reference; arrays are (count, pointer) pairs; every input is copied, no pointer is kept.
 * Quantities arrive canonical: cpu as MilliValue(), everything else as Value() (resource.Quantity
 * rounding, pkg/api/resource/quantity.go). */
#ifndef KSIM_K8S_H
#define KSIM_K8S_H

#include "ksim.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  const char* key;
  const char* value;
} ksim_k8s_kv;

/* A selector requirement: operator as the API spells it ("In", "NotIn", "Exists",
 * "DoesNotExist", "Gt", "Lt"; "=", "==", "!=" in resolved label selectors). */
typedef struct {
  const char* key;
  const char* op;
  int32_t n_values;
  const char* const* values;
} ksim_k8s_req;

/* v1.NodeSelectorTerm (its matchExpressions). */
typedef struct {
  int32_t n_reqs;
  const ksim_k8s_req* reqs;
} ksim_k8s_node_term;

/* v1.PreferredSchedulingTerm. */
typedef struct {
  int32_t weight;
  ksim_k8s_node_term preference;
} ksim_k8s_pref_node_term;

/* metav1.LabelSelector; present = 0 is a nil selector. */
typedef struct {
  int32_t present;
  int32_t n_match_labels;
  const ksim_k8s_kv* match_labels;
  int32_t n_exprs;
  const ksim_k8s_req* exprs;
} ksim_k8s_label_selector;

/* v1.PodAffinityTerm (weight: WeightedPodAffinityTerm.weight for preferred terms, else 0). */
typedef struct {
  ksim_k8s_label_selector selector;
  int32_t n_namespaces;
  const char* const* namespaces;
  const char* topology_key;
  int32_t weight;
} ksim_k8s_pod_term;

typedef struct {
  const char* key;
  const char* value;
  const char* effect;
} ksim_k8s_taint;

typedef struct {
  const char* key;
  const char* op;     /* "", "Equal" or "Exists" */
  const char* value;
  const char* effect;
} ksim_k8s_toleration;

typedef struct {
  const char* name;
  int64_t value;      /* Quantity.Value() */
} ksim_k8s_resource;

typedef struct {
  const char* host_ip;   /* "" / NULL: 0.0.0.0 */
  const char* protocol;  /* "" / NULL: TCP */
  int32_t host_port;     /* <= 0: not a host port */
} ksim_k8s_port;

/* One container's requests (and whether a cpu / memory request or limit is positive, for the
 * QoS class, K/pkg/apis/core/v1/helper/qos/qos.go:39-85). */
typedef struct {
  int32_t has_cpu, has_mem;          /* the requests map names cpu / memory */
  int64_t cpu_milli, mem, gpu, eph;  /* requests (0 when absent) */
  int32_t n_other;                   /* other requested resources (scalar ones are kept) */
  const ksim_k8s_resource* other;
  int32_t qos_positive;              /* some cpu / memory request or limit is > 0 */
  int32_t n_ports;
  const ksim_k8s_port* ports;
  const char* image;                 /* container.image (ImageLocalityPriority), NULL / "": none */
} ksim_k8s_container;

#define KSIM_K8S_VOL_GCE_PD 1
#define KSIM_K8S_VOL_EBS 2
#define KSIM_K8S_VOL_AZURE_DISK 3
#define KSIM_K8S_VOL_ISCSI 4
#define KSIM_K8S_VOL_RBD 5
#define KSIM_K8S_VOL_PVC 6
#define KSIM_K8S_VOL_OTHER 7

/* One volume: id = pdName / volumeID / diskName / iqn / claimName; RBD: monitors, pool, image. */
typedef struct {
  int32_t kind;
  int32_t read_only;
  const char* id;
  const char* pool;
  const char* image;
  int32_t n_monitors;
  const char* const* monitors;
} ksim_k8s_volume;

typedef struct {
  const char* name;
  const char* namespace_;
  int32_t n_labels;
  const ksim_k8s_kv* labels;
  int32_t deleting;                     /* metadata.deletionTimestamp is set */
  const char* node_name;                /* spec.nodeName, NULL / "": none */
  int32_t n_containers;
  const ksim_k8s_container* containers;
  int32_t n_init_containers;
  const ksim_k8s_container* init_containers;
  int32_t n_node_selector;
  const ksim_k8s_kv* node_selector;
  /* spec.affinity.nodeAffinity */
  int32_t has_node_affinity;
  int32_t has_required;                 /* requiredDuringSchedulingIgnoredDuringExecution is set */
  int32_t n_required_terms;
  const ksim_k8s_node_term* required_terms;
  int32_t n_preferred;
  const ksim_k8s_pref_node_term* preferred;
  int32_t n_tolerations;
  const ksim_k8s_toleration* tolerations;
  /* spec.affinity.podAffinity / podAntiAffinity */
  int32_t has_pod_affinity, has_pod_anti_affinity;
  int32_t n_affinity_required, n_affinity_preferred, n_anti_required, n_anti_preferred;
  const ksim_k8s_pod_term* affinity_required;
  const ksim_k8s_pod_term* affinity_preferred;
  const ksim_k8s_pod_term* anti_required;
  const ksim_k8s_pod_term* anti_preferred;
  int32_t n_volumes;
  const ksim_k8s_volume* volumes;
  /* getSelectors (priorities/metadata.go:82-114) as the caller's listers resolve it: the
   * selectors of the services / RCs (set_selector = 1: labels.SelectorFromSet over matchLabels)
   * and ReplicaSets / StatefulSets (0: LabelSelectorAsSelector) selecting the pod, in lister order */
  int32_t n_spread;
  const ksim_k8s_label_selector* spread;
  const int32_t* spread_set_selector;
  /* the RC / RS controllerRef NodePreferAvoidPods compares (kind, uid), NULL kind: none */
  const char* avoid_ctrl_kind;
  const char* avoid_ctrl_uid;
  const char* uid;                      /* metadata.uid: the cache's pod key (getPodKey, node_info.go:497-503);
                                           NULL / "": namespace/name */
} ksim_k8s_pod;

typedef struct {
  const char* type;
  const char* status;
} ksim_k8s_condition;

/* preferAvoidPods entry as v1helper.GetAvoidPodsFromNodeAnnotations decodes it; has_controller = 0
 * for an entry whose podSignature.podController is nil. */
typedef struct {
  int32_t has_controller;
  const char* kind;
  const char* uid;
} ksim_k8s_avoid;

/* v1.ContainerImage of status.images. */
typedef struct {
  int32_t n_names;
  const char* const* names;
  int64_t size_bytes;
} ksim_k8s_image;

typedef struct {
  const char* name;
  int32_t n_labels;
  const ksim_k8s_kv* labels;
  int32_t n_taints;
  const ksim_k8s_taint* taints;
  int32_t unschedulable;
  int32_t n_conditions;
  const ksim_k8s_condition* conditions;
  int64_t alloc_cpu_milli, alloc_mem, alloc_gpu, alloc_eph, alloc_pods;
  int32_t n_alloc_other;                /* other allocatable resources (scalar ones are kept) */
  const ksim_k8s_resource* alloc_other;
  int32_t n_avoid;
  const ksim_k8s_avoid* avoid;
  int32_t has_images;                   /* status.images is non-empty (implied by n_images > 0) */
  int32_t n_images;                     /* status.images (ImageLocalityPriority, image_locality.go:39-88) */
  const ksim_k8s_image* images;
} ksim_k8s_node;

typedef struct {
  const char* name;
  int32_t n_labels;
  const ksim_k8s_kv* labels;
  int32_t kind;                         /* KSIM_K8S_VOL_GCE_PD / _EBS / _AZURE_DISK / _OTHER */
  const char* id;
  int32_t has_node_affinity;
} ksim_k8s_pv;

typedef struct {
  const char* namespace_;
  const char* name;
  const char* volume_name;              /* spec.volumeName, "" / NULL: unbound */
  const char* storage_class;            /* spec.storageClassName, NULL: unset */
} ksim_k8s_pvc;

typedef struct {
  const char* name;
  const char* binding_mode;             /* volumeBindingMode, NULL: unset */
} ksim_k8s_storage_class;

typedef struct {
  int32_t hard_weight;                  /* hardPodAffinitySymmetricWeight (the simulator's 10) */
  int32_t max_vols[3];                  /* MaxPD limits (EBS, GCE PD, Azure Disk); 0: getMaxVols */
  int32_t port_slots;                   /* host-port slots per node, < 0: enough for the queue */
  int32_t vol_slots;                    /* volume slots per node, < 0: enough for the queue */
  int32_t image_locality;               /* intern node / pod images (what ImageLocalityPriority reads):
                                           0 = when some node lists status.images, 1 = always, -1 = never */
} ksim_k8s_options;

typedef struct ksim_k8s_cluster ksim_k8s_cluster;

/* A snapshot under construction: nodes, PVs / PVCs / storage classes, running pods (spec.nodeName
 * set) and the queue in scheduling order. */
int ksim_k8s_create(const ksim_k8s_options* opt, ksim_k8s_cluster** out);
void ksim_k8s_destroy(ksim_k8s_cluster* c);
const char* ksim_k8s_last_error(const ksim_k8s_cluster* c);
int ksim_k8s_add_node(ksim_k8s_cluster* c, const ksim_k8s_node* n);
int ksim_k8s_add_pv(ksim_k8s_cluster* c, const ksim_k8s_pv* pv);
int ksim_k8s_add_pvc(ksim_k8s_cluster* c, const ksim_k8s_pvc* pvc);
int ksim_k8s_add_storage_class(ksim_k8s_cluster* c, const ksim_k8s_storage_class* sc);
int ksim_k8s_add_running_pod(ksim_k8s_cluster* c, const ksim_k8s_pod* p);
int ksim_k8s_add_queued_pod(ksim_k8s_cluster* c, const ksim_k8s_pod* p);

/* Intern everything and build the tables (NodeInfo.SetNode / AddPod for the running pods, the
 * class, affinity and volume tables, the pod descriptors).  KSIM_E_UNSUPPORTED where the reference
 * errs instead of placing (ksim_k8s_last_error says which input). */
int ksim_k8s_build(ksim_k8s_cluster* c);

/* The configured scheduler on the built snapshot: cfg as for ksim_create (predicate bits and
 * priority weights; KSIM_W_SELECTOR_SPREAD carries SelectorSpread / ServiceSpreading's weight when
 * some pod has spread selectors), prefer_avoid_weight: NodePreferAvoidPodsPriority's weight (0: not
 * configured; it is the constant 10 x weight of cfg->const_score unless the nodes' preferAvoidPods
 * annotations tell some pod class apart).  Creates the handle and loads the node table, class /
 * affinity / volume tables and the queue. */
int ksim_k8s_open(ksim_k8s_cluster* c, const ksim_config* cfg, int64_t prefer_avoid_weight, ksim_handle** out);

/* Weights of the priorities the front end evaluates per (pod class, label set) on the host — they
 * have no ksim_config weight slot; 0 = not configured. */
typedef struct {
  int64_t prefer_avoid;   /* NodePreferAvoidPodsPriority (node_prefer_avoid_pods.go:32-68) */
  int64_t image_locality; /* ImageLocalityPriority (image_locality.go:39-88): with images interned
                             (ksim_k8s_options.image_locality), node images x pod container images;
                             KSIM_E_UNSUPPORTED when some node lists images the snapshot did not intern */
} ksim_k8s_weights;

/* ksim_k8s_open for a policy that may weigh ImageLocalityPriority; ksim_k8s_open(c, cfg, w_pa, out) is
 * ksim_k8s_open_ex with {w_pa, 0}: a policy without ImageLocalityPriority. */
int ksim_k8s_open_ex(ksim_k8s_cluster* c, const ksim_config* cfg, const ksim_k8s_weights* w, ksim_handle** out);

/* A Policy's keys with arguments (factory/plugins.go RegisterCustomFitPredicate /
 * RegisterCustomPriorityFunction over api.PredicateArgument / PriorityArgument):
 *  - CheckNodeLabelPresence (KSIM_P_LABEL_PRESENCE; predicates.go:875-910): every listed label present
 *    (presence = 1) or absent (0) on the node;
 *  - CheckServiceAffinity (KSIM_P_SERVICE_AFFINITY; predicates.go:940-1016) with the ServiceLister
 *    selecting none of the pods: the node must carry the pod's nodeSelector values of the labels;
 *  - labelPreference priorities (node_label.go:42-58): MaxPriority x weight when the label's
 *    presence on the node equals `presence`; a serviceAntiAffinity priority with no service selecting
 *    the pods (selector_spreading.go:221-275) is {label, presence = 1, weight}.  Label priorities
 *    have no ksim_config weight slot, but they ARE prioritizers: a Policy that configures only them
 *    must still pass cfg.no_priorities = 0 (the library fails with KSIM_E_INVAL otherwise).
 * services_select_pods: the adapter's ServiceLister selects some pod — CheckServiceAffinity and
 * serviceAntiAffinity then need the service-aware tables the Python host builds (KSIM_E_UNSUPPORTED). */
typedef struct {
  const char* label;
  int32_t presence;
  int32_t pad;
  int64_t weight;
} ksim_k8s_label_priority;

typedef struct {
  int32_t n_presence_labels;
  int32_t presence;
  const char* const* presence_labels;
  int32_t n_affinity_labels;
  int32_t services_select_pods;
  const char* const* affinity_labels;
  int32_t n_label_priorities;
  int32_t has_service_anti_affinity;    /* some label priority stands for a serviceAntiAffinity one */
  const ksim_k8s_label_priority* label_priorities;
} ksim_k8s_policy_args;

/* ksim_k8s_open_ex with a Policy's arguments (NULL: none — CheckNodeLabelPresence /
 * CheckServiceAffinity in cfg->predicates are then refused as before). */
int ksim_k8s_open_policy(ksim_k8s_cluster* c, const ksim_config* cfg, const ksim_k8s_weights* w,
                         const ksim_k8s_policy_args* args, ksim_handle** out);

/* Name-rank order and sizes of the built snapshot. */
int64_t ksim_k8s_node_count(const ksim_k8s_cluster* c);
const char* ksim_k8s_node_name(const ksim_k8s_cluster* c, int64_t rank);
int64_t ksim_k8s_queue_length(const ksim_k8s_cluster* c);

/* Built tables, read back (the parity tests compare them with the Python host's): the queued
 * pods' descriptors and their port / scalar arrays, a node's label-set / taint-set ids, a class
 * verdict: kind 0 = podMatchesNodeLabels bit of (class, label set), 1 = NoSchedule+NoExecute
 * tolerated (class, taint set), 2 = NoExecute tolerated, 3 = intolerable PreferNoSchedule count
 * (class, taint set), 4 = preferred node-affinity weight (class, label set). */
int ksim_k8s_pods(const ksim_k8s_cluster* c, const ksim_pod** pods, const uint64_t** ports, int64_t* n_ports,
                  const ksim_scalar_req** scalars, int64_t* n_scalars);
int ksim_k8s_node_sets(const ksim_k8s_cluster* c, int64_t rank, int32_t* label_set, int32_t* taint_set, uint32_t* flags);
int64_t ksim_k8s_class_value(const ksim_k8s_cluster* c, int32_t kind, int32_t cls, int32_t set);

/* The built tables as the structs ksim_load_nodes / _classes / _affinity / _volumes take (views
 * into the cluster, valid until the next call that changes it; absent tables are zeroed). */
int ksim_k8s_tables(ksim_k8s_cluster* c, ksim_node_table* nodes, ksim_class_tables* classes, ksim_affinity_tables* aff,
                    ksim_volume_tables* vol);

/* Per-pod drop-in (scheduler.go:188-204 scheduleOne): describe one more pod against an open
 * handle — its class, identity, affinity and volume classes interned, and the tables reloaded when
 * it brings new ones — ready for ksim_schedule_one; ports / scalars receive its arrays (capacity
 * given, counts returned).  ksim_k8s_bind records a placed pod (Scheduler.assume / cache.AddPod) so
 * later reloads keep its affinity counts and volume mounts. */
int ksim_k8s_describe(ksim_k8s_cluster* c, ksim_handle* h, const ksim_k8s_pod* p, ksim_pod* out, uint64_t* ports,
                      int32_t port_cap, int32_t* n_ports, ksim_scalar_req* scalars, int32_t scalar_cap,
                      int32_t* n_scalars, int64_t* pod_id);
int ksim_k8s_bind(ksim_k8s_cluster* c, int64_t pod_id, int64_t node);
/* The snapshot's per-pod path follows bindings only: once a node or pod event has reached the handle
 * directly (ksim_node_* / ksim_pod_*), describe refuses with KSIM_E_STATE rather than reload tables
 * from a stale view.  Event-driven callers use the scheduler cache below. */

/* ==== The scheduler cache: the complete per-pod drop-in ===================================
 * schedulercache.Cache (schedulercache/cache.go:125-393) + genericScheduler.Schedule
 * (core/generic_scheduler.go:112-198) over the device-resident table, driven by the informer events
 * the reference's config factory wires (factory/factory.go:596 addPodToCache, :613 updatePodInCache,
 * :695 deletePodFromCache, :740 addNodeToCache, :755 updateNodeInCache, :841 deleteNodeFromCache)
 * and by scheduleOne (scheduler.go:431-484: Schedule, assume = AssumePod, ForgetPod on a failed
 * bind, :412).  Every string rule is evaluated in the library; node rows, class / affinity / volume
 * tables grow or are reloaded as the events require.  The errors are cache.go's (KSIM_E_STATE, the
 * reference's message in ksim_k8s_cache_last_error); inputs the reference errs on are
 * KSIM_E_UNSUPPORTED, never a silently different placement. */
typedef struct ksim_k8s_cache ksim_k8s_cache;

typedef struct {
  ksim_config cfg;          /* device, mode, predicate bits, priority weights (ksim_create) */
  ksim_k8s_weights extra;   /* NodePreferAvoidPods / ImageLocality weights */
  int32_t hard_weight;      /* hardPodAffinitySymmetricWeight */
  int32_t max_vols[3];      /* MaxPD limits (EBS, GCE PD, Azure Disk); 0: getMaxVols */
  int32_t port_slots;       /* host-port slots per node row (<= 0: 8) */
  int32_t check_volume_binding; /* CheckVolumeBinding is configured (no kernel bit: refusals only) */
  int32_t pad;
  const ksim_k8s_policy_args* policy; /* a Policy's arguments (copied at create), NULL: none */
} ksim_k8s_cache_options;

int ksim_k8s_cache_create(const ksim_k8s_cache_options* opt, ksim_k8s_cache** out);
void ksim_k8s_cache_destroy(ksim_k8s_cache* c);
const char* ksim_k8s_cache_last_error(const ksim_k8s_cache* c);
/* the PV / PVC / StorageClass listers the volume predicates resolve PVCs through */
int ksim_k8s_cache_add_pv(ksim_k8s_cache* c, const ksim_k8s_pv* pv);
int ksim_k8s_cache_add_pvc(ksim_k8s_cache* c, const ksim_k8s_pvc* pvc);
int ksim_k8s_cache_add_storage_class(ksim_k8s_cache* c, const ksim_k8s_storage_class* sc);
/* node events: AddNode / UpdateNode → NodeInfo.SetNode (cache.go:354-375); RemoveNode (:378-393): the
 * node leaves the listed set, its NodeInfo stays while pods remain on it */
int ksim_k8s_cache_add_node(ksim_k8s_cache* c, const ksim_k8s_node* node);
int ksim_k8s_cache_update_node(ksim_k8s_cache* c, const ksim_k8s_node* old_node, const ksim_k8s_node* new_node);
int ksim_k8s_cache_remove_node(ksim_k8s_cache* c, const ksim_k8s_node* node);
/* pod events (pod->node_name = the node it is bound / assumed to): AssumePod (:125-143), ForgetPod
 * (:170-197), AddPod (:230-262, confirms an assumed pod), UpdatePod (:265-289), RemovePod (:292-318) */
int ksim_k8s_cache_assume_pod(ksim_k8s_cache* c, const ksim_k8s_pod* pod);
int ksim_k8s_cache_forget_pod(ksim_k8s_cache* c, const ksim_k8s_pod* pod);
int ksim_k8s_cache_add_pod(ksim_k8s_cache* c, const ksim_k8s_pod* pod);
int ksim_k8s_cache_update_pod(ksim_k8s_cache* c, const ksim_k8s_pod* old_pod, const ksim_k8s_pod* new_pod);
int ksim_k8s_cache_remove_pod(ksim_k8s_cache* c, const ksim_k8s_pod* pod);
/* genericScheduler.Schedule over the listed nodes; assume = KSIM_SCHEDULE_ASSUME also runs
 * Scheduler.assume (the pod enters the cache on the chosen node as an assumed pod).  KSIM_OK with
 * out->node = the host's name rank (ksim_k8s_cache_node_name), or -1 for a FitError
 * (ksim_k8s_cache_fit_error gives its text); KSIM_E_NO_NODES when no node is listed. */
int ksim_k8s_cache_schedule(ksim_k8s_cache* c, const ksim_k8s_pod* pod, int32_t assume, ksim_result* out);
/* FitError.Error of a result (generic_scheduler.go:72-90) into buf (NUL-terminated, truncated to cap);
 * returns the full length. */
int32_t ksim_k8s_cache_fit_error(const ksim_k8s_cache* c, const ksim_result* res, char* buf, int32_t cap);
int64_t ksim_k8s_cache_node_count(const ksim_k8s_cache* c);
const char* ksim_k8s_cache_node_name(const ksim_k8s_cache* c, int64_t rank);
/* the cache's scheduling handle (ksim_get_counter, ksim_read_nodes, ...); owned by the cache */
ksim_handle* ksim_k8s_cache_handle(ksim_k8s_cache* c);
/* counters of table work: [0] affinity loads, [1] volume loads, [2] volume grows, [3] class loads */
int ksim_k8s_cache_stats(const ksim_k8s_cache* c, int64_t* out4);

#ifdef __cplusplus
}
#endif

#endif /* KSIM_K8S_H */
