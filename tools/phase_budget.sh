#!/bin/bash
# Per-phase instruction budget of k_step (GPU box): step time and SQ counters
# of the product build and of the timing-only builds stopped after cars_pre (stop0), the car
# part (stop1), LiDAR phase 1 (stop2), phase 2 (stop3) and phase 3 (stop4).
# Differences between consecutive rows are the phases' costs.
set -e
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/ab_bench.sh stop0 stop1 stop2 stop3 stop4 ""
for v in stop0 stop1 stop2 stop3 stop4 ""; do
  rm -rf gpurun_out/sqb
  MEV_LIB_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
      SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/sqb -o run --output-format csv -- \
      python3 bench.py --no-kernel-events --no-cpu-baseline --no-gather --steps 100 --warmup 20 > gpurun_out/sqb.log 2>&1
  echo "== ${v:-product}"
  python tools/pmc_sq.py gpurun_out/sqb | grep -A9 k_step | grep "per wave"
done
