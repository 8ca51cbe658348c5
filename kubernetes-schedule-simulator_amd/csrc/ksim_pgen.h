// ksim_pgen.h — host/device interface of the general persistent kernel (ksim_pgen.hip): pods with
// inter-pod affinity, SelectorSpread, volumes or CheckServiceAffinity in one launch per call.
#pragma once
#include "ksim_common.h"

// Arguments beyond the context.  The affinity / volume descriptors travel by value (kernel
// arguments stay in scalar registers / the constant cache instead of being re-read from HBM after
// every barrier); the LDS layout is planned on the host (ksim_pgen_plan).
struct PGenArgs {
  uint64_t* gran;     // exchange: pass-A records, class granules, commit words (PG_* in ksim_pgen.hip)
  int32_t* cnt_row;   // [n_pair][n] row-form counted pairs
  int64_t* car_row;   // [n_carry][n] row-form carried terms
  const uint8_t* ident_shared;   // [n_ident] the identity's counted pairs include a shared-domain key
  const uint8_t* aclass_shared;  // [n_aclass] the class carries a term on a shared-domain key
  KsimAff A;          // valid when has_aff
  KsimVol V;          // valid when has_vol
  int32_t has_aff, has_vol;
  int32_t n_zone;     // zones of the spread reduce (<= PG_MAXZ)
  int32_t vs;         // volume slots staged per row in LDS (0: read from HBM)
  int32_t st_classes; // pod classes of the staged static (class, row) words (0: not staged)
  int32_t pad;
  uint64_t spin_ticks;
};

extern "C" hipError_t ksim_launch_pgen(const KsimCtx* c, const PGenArgs* g, int grid, int npt, hipStream_t s);
extern "C" int ksim_pgen_config(int64_t n, int max_grid, int* grid, int* npt);
// LDS plan for rows per workgroup `chunk`: volume slots staged per row and whether the static
// (class, row) words fit; returns the dynamic LDS bytes.
extern "C" size_t ksim_pgen_plan(int64_t chunk, int32_t n_classes, int32_t vol_slots, int32_t* vs, int32_t* st_classes);
extern "C" size_t ksim_pgen_gran_bytes(void);
extern "C" int ksim_pgen_max_zones(void);
extern "C" hipError_t ksim_pgen_rows(const KsimAff* aff_dev, int32_t* cnt_row, int64_t* car_row, int32_t n_pair,
                                     int32_t n_carry, int64_t n, int to_rows, hipStream_t s);
