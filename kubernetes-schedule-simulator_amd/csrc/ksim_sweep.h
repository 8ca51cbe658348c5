// ksim_sweep.h — kernel arguments of the scenario-sweep kernel (ksim_sweep.hip), shared with
// the host runtime.
#pragma once
#include "ksim_f64.h"

struct SwArgs {
  int64_t n;
  int32_t n_pods, scen0;
  const double* dac;  // static columns [n]
  const double* dam;
  const double* yc;
  const double* ym;
  const int32_t* allowed;
  const uint32_t* flags;
  double* rc;         // dynamic columns [S][n]
  double* rm;
  double* zc;
  double* zm;
  int32_t* count;
  const kf64::FPod* pods;  // [n_pods]
  const int32_t* w;        // [S][3]: LeastRequested, MostRequested, BalancedResourceAllocation
  uint32_t preds;
  int32_t no_prio;
  uint64_t counter0;
  int32_t* out_node;      // [S][n_pods]
  uint64_t* out_counter;  // [S]
};

#define KSIM_SWEEP_MAX_NODES 76800  // uint16 evaluations of one scenario in LDS (150 KiB)
