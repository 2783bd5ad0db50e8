#!/bin/bash
# PMC passes over output_conv1 (tools/conv_only.py) for one library
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
L=$1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pc_1 -o run -- python3 tools/conv_only.py $L 2 > gpurun_out/pc_1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pc_2 -o run -- python3 tools/conv_only.py $L 2 > gpurun_out/pc_2.log 2>&1 || exit 1
echo pmc done
