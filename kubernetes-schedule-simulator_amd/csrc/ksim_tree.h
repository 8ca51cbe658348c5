// ksim_tree.h — geometry of the per-pod-class selection trees (tree mode, ksim_tree.hip),
// shared by the kernels and the host runtime.
//
// Tree mode replaces the per-pod O(N) scan by an incremental
// tournament over the node table, for map-only policies and resource-only pods: between two
// pods only the committed node's row changes, so for every pod class only one leaf-to-root
// path of that class's tree changes.  Pods with identical predicate / priority inputs
// (GetResourceRequest, non-zero requests, BestEffort, "any request") share a class.
//
// Level 0 (leaves): int32 per (class, node) = -1 if the node fails the class's predicates,
// else its weighted map score.  Level h >= 1: one u64 per entry, (max score + 1) << 32 | the
// number of leaves below at that score (0 when nothing below fits), over its children (G0 =
// 64 m leaves for level 1, 64 entries above).  The root answers PrioritizeNodes' maximum and
// selectHost's count at the maximum, a per-class fit count kept beside it findNodesThatFit's
// len(filtered); selectHost's ix-th node from the top (descending name rank among the
// max-score nodes) is found by walking down the tree.
#pragma once
#include <stdint.h>

#define KSIM_TREE_MAX_CLASSES 64  /* one lane per class */
#define KSIM_TREE_MAX_LEVELS 8

struct KsimTreeGeo {
  int64_t n;                              // nodes (leaves per class)
  int32_t K;                              // tree classes
  int32_t m;                              // leaves per lane at the leaf level (G0 = 64 m)
  int32_t H;                              // internal levels 1..H (level H has one entry)
  int32_t hL;                             // levels hL..H are kept in LDS during a call
  int64_t nh[KSIM_TREE_MAX_LEVELS + 1];   // entries per class at level h (nh[0] = n)
  int64_t st[KSIM_TREE_MAX_LEVELS + 1];   // padded per-class stride of level h
  int64_t goff[KSIM_TREE_MAX_LEVELS + 1]; // offset of level h (h >= 1) in the global level array
  int32_t loff[KSIM_TREE_MAX_LEVELS + 1]; // offset of level h (h >= hL) in the LDS level array
  int64_t lds_entries;                    // u64 entries of the LDS levels
  int64_t level_entries;                  // u64 entries of the global level array
};

// The per-class predicate / priority inputs of a resource-only pod (kf64::FPod without the
// commit deltas, which stay per pod).
struct KsimTreeClass {
  double rq_c, rq_m, nz_c, nz_m;
  uint32_t anyreq, be;
};

// Scenario sweep through the trees (ksim_sweep): nsc independent copies of the cluster, each
// with its own dynamic columns ([nsc][n]), counter, map weights (kf64::EvCfg, opaque here) and
// output row of count_pods placements; trees laid out [nsc][...] in the same buffers.
struct KsimTreeSweep {
  int32_t nsc;
  int64_t count_pods;
  int64_t *rc, *rm, *zc, *zm;
  int32_t* count;
  uint64_t* counter;
  int32_t* out_node;
  const void* cfg;
};

#ifdef __cplusplus
extern "C" {
#endif
// Plans the tree for n nodes and K classes within lds_budget bytes (0 = default); returns 0
// when the table is beyond the tree's limits (more than 2^24 - 1 nodes, too many levels).
int ksim_tree_plan(int64_t n, int32_t K, int64_t lds_budget, int32_t force_m, KsimTreeGeo* g);
#ifdef __cplusplus
}
#endif
