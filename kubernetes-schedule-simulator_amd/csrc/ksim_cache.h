// ksim_cache.h — layouts shared by the scheduler-cache kernels (ksim_cache.hip) and their host
// side (ksim_cache.cpp): the node-table relayout used by node add / remove and port-slot growth,
// and the packed node row used by add / update.
#pragma once
#include <stdint.h>

#define KSIM_MAX_COLS 24

// One node column: `src_slots` slot-major [slot][n_old] rows of esz bytes in, `dst_slots`
// [slot][n_new] rows out (slots beyond src_slots, and an inserted row, are zero).
struct KsimRelayCol {
  const void* src;
  void* dst;
  int32_t esz;
  int32_t src_slots;
  int32_t dst_slots;
  int32_t pad;
};

#define KSIM_RELAY_SAME 0    /* same rows (slot growth) */
#define KSIM_RELAY_INSERT 1  /* a zero row appears at idx; rows >= idx move up one */
#define KSIM_RELAY_REMOVE 2  /* row idx disappears; rows > idx move down one */

struct KsimRelayout {
  KsimRelayCol col[KSIM_MAX_COLS];
  int32_t ncol;
  int32_t op;
  int64_t n_old, n_new, idx;
};

// Packed node row (u64 words): the ksim_node_row fields in a fixed order, then n_scalar
// allocatable scalars, n_scalar requested scalars and port_slots port keys.
#define KSIM_PK_ALLOC 0     /* 4 words: cpu, memory, gpu, ephemeral */
#define KSIM_PK_ALLOWED 4
#define KSIM_PK_FLAGS 5
#define KSIM_PK_LABEL 6
#define KSIM_PK_TAINT 7
#define KSIM_PK_REQ 8       /* 4 words: cpu, memory, gpu, ephemeral */
#define KSIM_PK_NZ 12       /* 2 words: cpu, memory */
#define KSIM_PK_COUNT 14
#define KSIM_PK_PORTCNT 15
#define KSIM_PK_SCALAR 16
#define KSIM_PK_WORDS(n_scalar, port_slots) (KSIM_PK_SCALAR + 2 * (n_scalar) + (port_slots))
