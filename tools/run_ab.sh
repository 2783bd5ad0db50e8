#!/bin/bash
# A/B of the encoder GEMMs: in-tree phased vs the 2-blocks-per-CU kernel (2 and 1 block per CU).
set -o pipefail
python -c "
import ctypes; l=ctypes.CDLL('build/g2/libvda_c.so'); import torch; torch.zeros(1,device='cuda')
print('occupancy fc1/fc2 blocks per CU:', l.vda_debug_gemm2(99, 0))"
timeout -k 10 300 python tools/ab_gemm.py video-depth-anything_amd/libvda.so build/g2/libvda.so@g2=0 build/g2/libvda_b.so@g2m2=0 --rounds 5 --shapes fc2,fc1 > gpurun_out/ab_gemm.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_gemm.log; exit $rc
