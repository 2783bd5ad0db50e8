set -o pipefail
timeout -k 10 300 python bench.py > gpurun_out/base_bench.log 2>&1 && tail -1 gpurun_out/base_bench.log | cut -c1-600 &&
timeout -k 10 200 python tools/bench_gemm.py 4 > gpurun_out/base_gemm.log 2>&1; tail -12 gpurun_out/base_gemm.log
