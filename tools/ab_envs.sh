#!/bin/bash
# k_step time per step (bench.py stream events, kernel events off) for library
# variants at several batch sizes: bash tools/ab_envs.sh "1024 4096" "" variantA ...
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
envs=$1; shift
for e in $envs; do
  for v in "$@"; do
    printf "envs %5d variant %-10s " "$e" "${v:-product}"
    MEV_LIB_VARIANT=$v timeout -k 10 120 python bench.py --envs "$e" --no-cpu-baseline --no-gather --steps 1000 --warmup 50 --no-kernel-events --step-kernel ${STEPK:-2} |
      python -c "import json,sys; d=json.load(sys.stdin); print(round(d['ms_per_step']*1e3,2), 'us/step', round(d['value']/1e6,1), 'M agent-steps/s')"
  done
done
