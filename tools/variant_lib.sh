#!/bin/bash
# Diagnostic A/B builds: libksim.so with ksim_pfast.hip replaced by another source (and/or extra
# defines), linked with the product objects of csrc/build, into lib/<name>/libksim.so.
# Usage: tools/variant_lib.sh <name> <pfast source> [extra hipcc flags...]   (run here, on the CPU)
set -e
NAME=$1; SRC=$(realpath "$2"); shift 2
cd "$(dirname "$0")/../kubernetes-schedule-simulator_amd/csrc"
make -s >/dev/null
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Wno-unused-function"
mkdir -p ../lib/$NAME build/v_$NAME
cp "$SRC" build/v_$NAME/ksim_pfast.hip
/opt/rocm/bin/hipcc $FLAGS -I. "$@" -c build/v_$NAME/ksim_pfast.hip -o build/v_$NAME/ksim_pfast.o
OBJS=$(ls build/*.o | grep -v ksim_pfast)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../lib/$NAME/libksim.so $OBJS build/v_$NAME/ksim_pfast.o
echo "built lib/$NAME/libksim.so"
