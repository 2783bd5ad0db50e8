#!/bin/bash
# attention PMC passes (a0 = kernel, a2 = pipelined variant) + per-phase tile timestamps of the GEMMs
set -o pipefail
bash tools/pmc_attn.sh build/var/a0/libvda.so build/var/a2/libvda.so || exit 1
timeout -k 10 200 python tools/ts_probe2.py build/ts/libvda.so qkv,fc1,proj,fc2 > gpurun_out/ts3.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/ts3.log | head -40
