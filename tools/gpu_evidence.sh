#!/bin/bash
# Round evidence on the GPU box: GPU tests, bench line, rocprofv3 kernel stats, the
# SQ (VALU) counter pass, the two PMC traffic passes and the config sweep. Every GPU
# step has its own time limit; the first failure ends the script (set -e), nothing
# is retried.
# Usage (via gpurun): bash tools/gpu_evidence.sh [tests|bench|sweep|all]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out
mkdir -p $OUT
what=${1:-all}
if [ "$what" = tests ] || [ "$what" = all ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
    || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
  # SQ pass first: bench.py's roofline.valu reads profiles/valu_counters.json
  rm -rf $OUT/sq
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
      -d $OUT/sq -o run --output-format csv -- python3 bench.py --no-kernel-events --no-cpu-baseline --no-gather --steps 200 > $OUT/sq.log 2>&1
  python tools/valu_counters.py $OUT/sq --out $OUT/valu_counters.json > /dev/null
  cp $OUT/valu_counters.json profiles/valu_counters.json
  python tools/pmc_sq.py $OUT/sq > $OUT/sq_counters.txt
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf $OUT/pmc_$c
    timeout -s KILL 90 rocprofv3 --pmc $c -d $OUT/pmc_$c -o run --output-format csv -- \
      python3 bench.py --no-kernel-events --no-cpu-baseline --no-gather --steps 200 > $OUT/pmc_$c.log 2>&1
  done
  python tools/pmc_traffic.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE --envs 4096 --agents 8 --rays 64 --out $OUT/pmc_traffic.json > /dev/null
  cp $OUT/pmc_traffic.json profiles/pmc_traffic.json
  rm -rf $OUT/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python3 bench.py --no-kernel-events --no-cpu-baseline --no-gather > $OUT/prof_bench.log 2>&1
  find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
  cut -c1-200 $OUT/kernel_stats.csv
  timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
  cat $OUT/bench.json
  timeout -k 10 300 python bench.py --kernel-events --no-cpu-baseline > $OUT/bench_events.json 2>> $OUT/bench.err
fi
if [ "$what" = sweep ] || [ "$what" = all ]; then
  timeout -k 10 300 python tools/bench_sweep.py --out $OUT/sweep.json > $OUT/sweep.txt 2>&1
  tail -12 $OUT/sweep.txt
  timeout -k 10 300 python tools/env_latency.py > $OUT/env_latency.txt 2>&1
  tail -12 $OUT/env_latency.txt
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
  tail -2 $OUT/smoke.txt
fi
