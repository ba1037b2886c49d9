#!/bin/bash
# A/B of library variants on one bench_sweep config, interleaved (A B A B ...) so
# clock drift and box noise hit every variant alike:
#   bash tools/ab_sweep.sh cfg4 ROUNDS "" variantA variantB ...   ("" = product)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cfg=$1; rounds=$2; shift 2
for r in $(seq "$rounds"); do
  for v in "$@"; do
    printf "round %d variant %-12s " "$r" "${v:-product}"
    MEV_LIB_VARIANT=$v timeout -k 10 120 python tools/bench_sweep.py --only "$cfg" --steps 1000 2>/dev/null |
      python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['agent_steps_per_s']/1e6,2), 'M agent-steps/s', round(d['ms_per_step']*1e3,2), 'us/step')"
  done
done
