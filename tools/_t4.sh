set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash tools/ab_sweep.sh cfg3 1 "" nohelp
bash tools/ab_sweep.sh cfg2 1 "" nohelp
bash tools/ab_sweep.sh cfg5 1 "" nohelp
