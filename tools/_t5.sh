set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/t5; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_parity_gpu.py tests/test_gpu_vs_oracle.py tests/test_properties_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for pk in 1 2 4; do
timeout -k 10 300 python tools/bench_sweep.py --only cfg2,cfg3 --pack $pk 2>/dev/null | grep name
done
