#!/bin/bash
# one PMC pass over the spatial attention of each library given (VALU / MFMA co-execution, waits)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for L in "$@"; do
  tag=$(basename $(dirname $L))
  timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pb_${tag} -o run -- python3 tools/attn_only.py $L 3 > gpurun_out/pb_${tag}.log 2>&1 || exit 1
done
echo pmc done
