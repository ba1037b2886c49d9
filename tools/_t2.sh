set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/t2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_gpu_vs_oracle.py tests/test_properties_gpu.py -m gpu -x -q -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep "sequential NPC" $O/pytest.log || true
tail -3 $O/pytest.log
for v in ""; do
MEV_LIB_VARIANT=$v timeout -k 10 300 python tools/bench_sweep.py --only cfg4 > $O/sweep_$v.txt 2>&1
echo "variant $v"; grep cfg4 $O/sweep_$v.txt
done
MEV_LIB_VARIANT=stamps timeout -k 10 200 python tools/npc_profile.py > $O/npc.txt 2>&1 || true
MEV_LIB_VARIANT=stampsn timeout -k 10 200 python tools/npc_profile.py --parts > $O/npc_parts.txt 2>&1 || true
cat $O/npc.txt $O/npc_parts.txt
