#!/bin/bash
# Builds escalator_amd/libescalator_hip_<NAME>.so: the library with esc_kernels.hip part 0
# compiled with extra flags (e.g. -DK1_PK_DS=8), for A/B timing through ESC_LIB_PATH.
set -e
NAME=$1; shift
cd "$(dirname "$0")/../escalator_amd/csrc"
B=../../build/var_$NAME
mkdir -p $B
HIPCC=/opt/rocm/bin/hipcc
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result -I../../include -I."
$HIPCC $FL "$@" -DESC_PART=0 -c esc_kernels.hip -o $B/esc_kernels.o
O=../../build/csrc
RT=$O/esc_runtime.o
if [ -n "$REBUILD_RT" ]; then            # flags that change the runtime's view too (e.g. -DESC_ORD_CHUNK)
    $HIPCC $FL "$@" -c esc_runtime.hip -o $B/esc_runtime.o
    RT=$B/esc_runtime.o
fi
$HIPCC --offload-arch=gfx950 -shared -fPIC -o ../libescalator_hip_$NAME.so $B/esc_kernels.o $RT \
    $O/esc_multi.o $O/esc_list.o $O/esc_pack.o $O/esc_synth.o -pthread
