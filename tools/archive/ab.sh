#!/bin/bash
# A/B on one box: alternate build/old/libvda.so and the in-tree lib, N rounds, given command.
# usage: tools/ab.sh ROUNDS CMD...
R=$1; shift
for i in $(seq 1 $R); do
  for L in build/old/libvda.so video-depth-anything_amd/libvda.so; do
    echo "== $L"; VDA_LIB_OVERRIDE=$L timeout -k 10 300 "$@" 2>&1 | grep -v amdgpu.ids
  done
done
