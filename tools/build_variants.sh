#!/bin/bash
# Build libvda variants of one source file with extra -D flags: build/var/<name>/libvda.so
# usage: [SRC=vda_gemm EXTRA="-fno-slp-vectorize"] tools/build_variants.sh name1:"-DFOO" name2:"-DBAR" ...
set -e
TD=$(python3 -c "import os, torch; print(os.path.dirname(torch.__file__))")
FL="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result -I include -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form"
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  D=build/var/$name; mkdir -p $D
  S=${SRC:-vda_depth}
  /opt/rocm/bin/hipcc $FL $defs $EXTRA -c video-depth-anything_amd/csrc/$S.hip -o $D/$S.o
  objs=$(ls build/*.o | grep -v "/$S.o" | grep -v "/vda_torch.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs $D/$S.o -o $D/libvda.so
  # the torch op library linked next to it (VDA_LIB_OVERRIDE=$D/libvda.so picks up both)
  g++ build/vda_torch.o -o $D/libvda_torch.so -shared -L $TD/lib -lc10 -lc10_hip -ltorch_cpu -ltorch_hip -ltorch \
    -L $D -lvda -Wl,-rpath,'$ORIGIN' -Wl,-rpath,$TD/lib
  echo "built $D ($defs)"
done
