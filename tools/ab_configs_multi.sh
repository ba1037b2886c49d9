#!/bin/bash
# Interleaved A/B of library variants over several bench_sweep configs:
#   bash tools/ab_configs_multi.sh ROUNDS "cfg2,cfg3,cfg4" "" variantA ...   ("" = product)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rounds=$1; cfgs=$2; shift 2
for r in $(seq "$rounds"); do
  for v in "$@"; do
    printf "round %d %-10s " "$r" "${v:-product}"
    MEV_LIB_VARIANT=$v timeout -k 10 300 python tools/bench_sweep.py --only "$cfgs" --steps 1000 2>/dev/null |
      python -c "
import json,sys
print('  '.join('%s %.1fM %.2fus' % (d['name'], d['agent_steps_per_s']/1e6, d['ms_per_step']*1e3) for d in map(json.loads, sys.stdin.read().strip().splitlines())))"
  done
done
