#!/bin/bash
# Round evidence on the GPU box: GPU tests, bench line, rocprofv3 kernel stats and
# the two PMC traffic passes. Every GPU step has its own time limit; the first
# failure ends the script (set -e + &&), nothing is retried.
# Usage (via gpurun): bash tools/gpu_evidence.sh [tests|bench|all]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out
mkdir -p $OUT
what=${1:-all}
if [ "$what" = tests ] || [ "$what" = all ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  tail -3 $OUT/pytest_gpu.log
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
  timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
  cat $OUT/bench.json
  timeout -k 10 300 python bench.py --no-kernel-events --no-cpu-baseline > $OUT/bench_noevents.json 2>> $OUT/bench.err
  rm -rf $OUT/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python3 bench.py --no-kernel-events --no-cpu-baseline > $OUT/prof_bench.log 2>&1
  rm -rf $OUT/pmc_fetch $OUT/pmc_write
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- \
      python3 bench.py --no-kernel-events --no-cpu-baseline --steps 200 > $OUT/pmc_fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- \
      python3 bench.py --no-kernel-events --no-cpu-baseline --steps 200 > $OUT/pmc_write.log 2>&1
  rm -rf $OUT/sq1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
      -d $OUT/sq1 -o run --output-format csv -- python3 bench.py --no-kernel-events --no-cpu-baseline --steps 200 > $OUT/sq1.log 2>&1
  python tools/pmc_sq.py $OUT/sq1 > $OUT/sq_counters.txt
  find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
  cat $OUT/kernel_stats.csv | cut -c1-200
fi
