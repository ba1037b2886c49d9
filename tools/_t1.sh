set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/t1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_properties_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python tools/bench_sweep.py --only cfg4 > $O/sweep_auto.txt 2>&1
timeout -k 10 300 python tools/bench_sweep.py --only cfg4 --step-kernel 1 > $O/sweep_k1.txt 2>&1
cat $O/sweep_*.txt | grep -v amdgpu
MEV_LIB_VARIANT=stamps timeout -k 10 200 python tools/npc_profile.py > $O/npc.txt 2>&1 || true
cat $O/npc.txt
