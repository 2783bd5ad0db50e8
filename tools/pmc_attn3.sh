#!/bin/bash
# two PMC passes over the spatial attention of each library given: wait / issue breakdown and
# MFMA / VALU co-execution (tuning tool).  usage: tools/pmc_attn3.sh LIB.so ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for L in "$@"; do
  tag=$(basename $(dirname $L))
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pw_${tag}_a -o run -- python3 tools/attn_only.py $L 3 > gpurun_out/pw_${tag}_a.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pw_${tag}_b -o run -- python3 tools/attn_only.py $L 3 > gpurun_out/pw_${tag}_b.log 2>&1 || exit 1
done
echo pmc done
