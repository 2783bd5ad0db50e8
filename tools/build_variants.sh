#!/bin/bash
# Build libvda variants of one source file with extra -D flags: build/var/<name>/libvda.so
# usage: tools/build_variants.sh name1:"-DFOO" name2:"-DBAR" ...
set -e
FL="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result -I include -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form"
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  D=build/var/$name; mkdir -p $D
  /opt/rocm/bin/hipcc $FL $defs -c video-depth-anything_amd/csrc/vda_depth.hip -o $D/vda_depth.o
  objs=$(ls build/*.o | grep -v vda_depth.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs $D/vda_depth.o -o $D/libvda.so
  echo "built $D ($defs)"
done
