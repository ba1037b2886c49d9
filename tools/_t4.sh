set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread 2>&1 | tail -1
bash tools/ab_sweep.sh cfg3 1 "" noearlypath
bash tools/ab_sweep.sh cfg2 1 "" noearlypath
bash tools/ab_sweep.sh cfg1 1 "" noearlypath
bash tools/ab_sweep.sh cfg4 1 "" noearlypath
