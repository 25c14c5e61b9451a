#!/bin/bash
# libdreamer_hip with the persistent unroll's stage timestamps (DR_PDREAM_TS):
# dream.hip and engine.hip (workspace size) recompiled, the other objects reused.
set -e
cd "$(dirname "$0")/.."
python -m dreamer_amd.build > /dev/null
O=tools/variants/_build_pdts
mkdir -p $O
FL="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-gpu-rdc -Wall -Wno-unused-function -Wno-unused-variable -DDR_PDREAM_TS=1"
/opt/rocm/bin/hipcc $FL -c dreamer_amd/csrc/dream.hip -o $O/dream.o &
/opt/rocm/bin/hipcc $FL -c dreamer_amd/csrc/engine.hip -o $O/engine.o &
wait
objs=$(ls dreamer_amd/_build/*.o | grep -v -e '/dream.o' -e '/engine.o')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/libdreamer_hip_pdts.so $O/dream.o $O/engine.o $objs
echo built tools/variants/libdreamer_hip_pdts.so
