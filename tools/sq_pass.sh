#!/bin/bash
# One SQ counter pass + the per-SIMD stamp timeline of the current k_step (GPU box).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out
rm -rf $OUT/sq
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  -d $OUT/sq -o run --output-format csv -- python3 bench.py --no-kernel-events --no-cpu-baseline --no-gather --steps 200 > $OUT/sq.log 2>&1
python tools/valu_counters.py $OUT/sq --out $OUT/valu_counters.json > /dev/null
python tools/pmc_sq.py $OUT/sq > $OUT/sq_counters.txt
cat $OUT/sq_counters.txt
for e in 4096 1024; do
  MEV_LIB_VARIANT=stampsr timeout -k 10 120 python tools/simd_balance.py --envs $e 2>&1 | grep -v amdgpu.ids
done
