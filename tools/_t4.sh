set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_lidar_stress_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread 2>&1 | tail -1
bash tools/ab_sweep.sh cfg3 2 "" nostraight
bash tools/ab_sweep.sh cfg2 2 "" nostraight
bash tools/ab_sweep.sh cfg4 1 "" nostraight
