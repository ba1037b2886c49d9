set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pack" > gpurun_out/pytest_pack.log 2>&1 || { tail -30 gpurun_out/pytest_pack.log; exit 1; }
tail -2 gpurun_out/pytest_pack.log
for r in 1 2; do
for pk in 2 4 8; do for sp in 1 2; do
  printf "pack %d split %d: " $pk $sp
  timeout -k 10 120 python tools/bench_sweep.py --only cfg2 --steps 1000 --pack $pk --split $sp 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['agent_steps_per_s']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us', d['envs_per_wave'], d['waves_per_workgroup'])"
done; done; done
