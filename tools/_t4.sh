set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_gpu_vs_oracle.py -k "traffic or npc or dense" -m gpu -x -q --timeout 180 --timeout-method thread 2>&1 | tail -1
bash tools/ab_sweep.sh cfg4 2 "" nofar
