set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash tools/ab_bench.sh ""
timeout -k 10 300 python tools/bench_sweep.py > gpurun_out/sweep.txt 2>&1; cat gpurun_out/sweep.txt | tail -12
