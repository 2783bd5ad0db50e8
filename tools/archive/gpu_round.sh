set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 && tail -1 gpurun_out/bench_default.log
timeout -k 10 300 python bench.py --video --steps 3 --warmup 1 > gpurun_out/bench_video.log 2>&1 && tail -1 gpurun_out/bench_video.log
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --cpu-baseline-frames 0 > gpurun_out/bench_gloo2.log 2>&1 && tail -1 gpurun_out/bench_gloo2.log
