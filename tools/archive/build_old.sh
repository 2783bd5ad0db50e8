#!/bin/bash
# Build build/old/libvda.so from a git revision's kernel sources (A/B baseline for tools/ab_prof.sh).
# usage: tools/build_old.sh [REV]   (default HEAD)
REV=${1:-HEAD}
set -e
D=build/old/src; rm -rf $D; mkdir -p $D/csrc $D/include
for f in $(git ls-tree --name-only $REV video-depth-anything_amd/csrc/); do git show $REV:$f > $D/csrc/$(basename $f); done
git show $REV:include/vda.h > $D/include/vda.h
FL="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result -I $D/include -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form"
sed -i 's|../../include/vda.h|vda.h|' $D/csrc/*.hip
OBJS=""
for f in $D/csrc/*.hip; do
  X=""; [ "$(basename $f)" = vda_attn.hip ] && X="-fno-honor-nans -mno-amdgpu-ieee"
  [ "$(basename $f)" = vda_gemm.hip ] && X="-fno-slp-vectorize"
  /opt/rocm/bin/hipcc $FL $X -I $D/include -c $f -o ${f%.hip}.o & OBJS="$OBJS ${f%.hip}.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS -o build/old/libvda.so
echo "build/old/libvda.so <- $REV"
