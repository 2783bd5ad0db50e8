set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -x -k "dynamic_tile or layernorm_fold_stress or epilogue_row_stats" --timeout 200 --timeout-method thread > gpurun_out/dyn_test.log 2>&1; rc=$?; tail -3 gpurun_out/dyn_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/gemm_lab/run_lab.py --variants 5,30,31,32,33,40,42,43,50,51 --shapes qkv,fc1,fc2,sq8k > gpurun_out/lab6.log 2>&1; cat gpurun_out/lab6.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --cpu-baseline-frames 0 --no-probe --tiles dynamic > gpurun_out/ab_dyn_$r.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --cpu-baseline-frames 0 --no-probe --tiles static > gpurun_out/ab_static_$r.log 2>&1 || exit 1
  echo "dyn $(grep -o '"value": [0-9.]*' gpurun_out/ab_dyn_$r.log)  static $(grep -o '"value": [0-9.]*' gpurun_out/ab_static_$r.log)"
done
