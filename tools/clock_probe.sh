#!/bin/bash
# Build the clock-probe libraries (tools/clock_probe.py): build/ts/libvda.so (-DVDA_TS stamps) and
# build/probe/libclockprobe.so (the MFMA-only / DMA-only probe kernels).
set -e
bash tools/build_ts.sh
mkdir -p build/probe
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 tools/clock_probe.hip -o build/probe/libclockprobe.so
echo "built build/probe/libclockprobe.so"
