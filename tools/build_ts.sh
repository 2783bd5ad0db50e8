#!/bin/bash
# Instrumented build for tools/ts_probe2.py / ts_hconv.py / ts_oc1.py / ts_dconv.py: build/ts/{libvda.so, libvda_torch.so} with -DVDA_TS in the GEMM, the halo-tiled conv, output_conv1, the depth conv and the spatial attention.
# usage: bash tools/build_ts.sh ; VDA_LIB_OVERRIDE=build/ts/libvda.so python tools/ts_probe2.py
set -e
FL="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result -I include -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form"
D=build/ts; mkdir -p $D
/opt/rocm/bin/hipcc $FL -fno-slp-vectorize -DVDA_TS -c video-depth-anything_amd/csrc/vda_gemm.hip -o $D/vda_gemm.o
/opt/rocm/bin/hipcc $FL -DVDA_TS -c video-depth-anything_amd/csrc/vda_hconv.hip -o $D/vda_hconv.o
/opt/rocm/bin/hipcc $FL -DVDA_TS -c video-depth-anything_amd/csrc/vda_depth.hip -o $D/vda_depth.o
/opt/rocm/bin/hipcc $FL -DVDA_TS -c video-depth-anything_amd/csrc/vda_dconv.hip -o $D/vda_dconv.o
/opt/rocm/bin/hipcc $FL -fno-honor-nans -mno-amdgpu-ieee -fno-slp-vectorize -DVDA_TS -c video-depth-anything_amd/csrc/vda_attn.hip -o $D/vda_attn.o
objs=$(ls build/*.o | grep -v "/vda_gemm.o" | grep -v "/vda_hconv.o" | grep -v "/vda_depth.o" | grep -v "/vda_dconv.o" | grep -v "/vda_attn.o" | grep -v "/vda_torch.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs $D/vda_gemm.o $D/vda_hconv.o $D/vda_depth.o $D/vda_dconv.o $D/vda_attn.o -o $D/libvda.so
TD=$(python3 -c "import os, torch; print(os.path.dirname(torch.__file__))")
g++ build/vda_torch.o -o $D/libvda_torch.so -shared -L $TD/lib -lc10 -lc10_hip -ltorch_cpu -ltorch_hip -ltorch \
  -L $D -lvda -Wl,-rpath,'$ORIGIN' -Wl,-rpath,$TD/lib
echo "built $D"
