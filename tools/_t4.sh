set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MEV_LIB_VARIANT=wblate timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_properties_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread 2>&1 | tail -2
bash tools/ab_sweep.sh cfg3 2 "" wblate
bash tools/ab_sweep.sh cfg2 2 "" wblate
