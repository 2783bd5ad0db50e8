#!/bin/bash
# WRITE_SIZE of the fc1 GEMM for each library given (tools/gemm_only.py, C ABI)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for L in "$@"; do
  tag=$(basename $(dirname $L))
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pw_${tag} -o run -- python3 tools/gemm_only.py $L fc1 3 > gpurun_out/pw_${tag}.log 2>&1 || exit 1
done
echo pmc done
