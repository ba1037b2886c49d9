#!/bin/bash
# SQ counter pass (VALU / SALU / LDS instructions, wave cycles) over bench_sweep configs
# other than bench.py's (GPU box): bash tools/sq_configs.sh cfg2 cfg4 ...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out
for c in "$@"; do
  d=$OUT/sq_$(echo "$c" | tr -c 'a-zA-Z0-9\n' '_')
  rm -rf "$d"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
    -d "$d" -o run --output-format csv -- python3 tools/bench_sweep.py --only "$c" --steps 200 > "$d.log" 2>&1
  echo "== $c"
  python tools/pmc_sq.py "$d"
done
