#!/bin/bash
# Builds libksim.so variants with a 512-cycle delay at critical-path probe point k (-DKSIM_PROBE=k)
# into kubernetes-schedule-simulator_amd/lib/probe<k>/ (diagnostic; run here, on the CPU).
# Usage: tools/probe_libs.sh k1 k2 ...
set -e
cd "$(dirname "$0")/../kubernetes-schedule-simulator_amd/csrc"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Wno-unused-function"
for k in "$@"; do
  mkdir -p ../lib/probe$k
  /opt/rocm/bin/hipcc $FLAGS -DKSIM_PROBE=$k -shared -o ../lib/probe$k/libksim.so ksim_kernels.hip ksim_persistent.hip \
    ksim_pfast.hip ksim_sweep.hip ksim_tree.hip ksim_cache.hip -x hip ksim_runtime.cpp ksim_cache.cpp ksim_affinity.cpp &
done
wait
