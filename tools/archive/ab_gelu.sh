set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gelu_tests.log 2>&1 && tail -3 gpurun_out/gelu_tests.log &&
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --cpu-baseline-frames 0 > gpurun_out/gelu_b1.log 2>&1 && tail -1 gpurun_out/gelu_b1.log | cut -c1-200 &&
VDA_LIB_OVERRIDE=$PWD/build/oldg/libvda.so timeout -k 10 240 python bench.py --steps 20 --warmup 5 --cpu-baseline-frames 0 > gpurun_out/gelu_b0.log 2>&1 && tail -1 gpurun_out/gelu_b0.log | cut -c1-200 &&
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --cpu-baseline-frames 0 > gpurun_out/gelu_b2.log 2>&1 && tail -1 gpurun_out/gelu_b2.log | cut -c1-200
