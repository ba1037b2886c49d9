#!/bin/bash
# A/B of library variants over several bench_sweep configs, interleaved per round:
#   bash tools/ab_configs.sh ROUNDS "cfg1,cfg2,cfg3" "" variantA ...   ("" = product)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rounds=$1; cfgs=$2; shift 2
for r in $(seq "$rounds"); do
  for v in "$@"; do
    MEV_LIB_VARIANT=$v timeout -k 10 200 python tools/bench_sweep.py --only "$cfgs" --steps 1000 2>/dev/null |
      python -c "
import json,sys
for l in sys.stdin.read().strip().splitlines():
    d=json.loads(l); print('round $r variant %-10s %-8s %9.2f M agent-steps/s %7.2f us/step' % ('${v:-product}', d['name'], d['agent_steps_per_s']/1e6, d['ms_per_step']*1e3))"
  done
done
