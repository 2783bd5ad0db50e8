#!/bin/bash
# two PMC passes over tools/conv_gemm_only.py (the halo conv and the dense GEMM side by side): issue / wait /
# LDS-conflict counters (tuning tool).  usage: tools/pmc_conv_gemm.sh LIB.so
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
L=$1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pcg_a -o run -- python3 tools/conv_gemm_only.py $L 3 > gpurun_out/pcg_a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pcg_b -o run -- python3 tools/conv_gemm_only.py $L 3 > gpurun_out/pcg_b.log 2>&1 || exit 1
echo pmc done
