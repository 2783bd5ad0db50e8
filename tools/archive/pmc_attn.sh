#!/bin/bash
# PMC passes over the spatial attention (tools/attn_only.py) for the libraries given; each pass its own run.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for L in "$@"; do
  tag=$(basename $(dirname $L))
  timeout -k 10 200 python tools/ab_attn.py $L > gpurun_out/pa_${tag}_time.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pa_${tag}_1 -o run -- python3 tools/attn_only.py $L 3 > gpurun_out/pa_${tag}_1.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pa_${tag}_2 -o run -- python3 tools/attn_only.py $L 3 > gpurun_out/pa_${tag}_2.log 2>&1 || exit 1
done
echo pmc done
