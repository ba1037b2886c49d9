set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/t4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_gpu_vs_oracle.py tests/test_properties_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab_sweep.sh cfg4 2 "" prev
for r in 1 2; do for pk in 2 4; do
printf "cfg2 pack %d " $pk; timeout -k 10 120 python tools/bench_sweep.py --only cfg2 --pack $pk --steps 1000 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['agent_steps_per_s']/1e6,2), d['envs_per_wave'])"
done; done
