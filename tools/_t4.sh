set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/t4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_gpu_vs_oracle.py tests/test_properties_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab_sweep.sh cfg4 2 "" noprefilter
