#!/bin/bash
# libdreamer_hip with the persistent BPTT's stage timestamps (DR_PBPTT_TS):
# bptt.hip and engine.hip (workspace size) recompiled, the other objects reused.
set -e
cd "$(dirname "$0")/.."
python -m dreamer_amd.build > /dev/null
O=tools/variants/_build_pbts
mkdir -p $O
FL="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-gpu-rdc -Wall -Wno-unused-function -Wno-unused-variable -DDR_PBPTT_TS=1"
/opt/rocm/bin/hipcc $FL -c dreamer_amd/csrc/bptt.hip -o $O/bptt.o &
/opt/rocm/bin/hipcc $FL -c dreamer_amd/csrc/engine.hip -o $O/engine.o &
wait
objs=$(ls dreamer_amd/_build/*.o | grep -v -e '/bptt.o' -e '/engine.o')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/libdreamer_hip_pbts.so $O/bptt.o $O/engine.o $objs
echo built tools/variants/libdreamer_hip_pbts.so
