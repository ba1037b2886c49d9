#!/bin/bash
# A/B timing of library variants on the GPU box (bench.py's config 3, kernel
# events off): bash tools/ab_bench.sh "" variantA variantB ...   ("" = product)
# Each variant is libmarlenv_hip_<name>.so next to the product library.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "$@"; do
  printf "variant %-10s " "${v:-product}"
  MEV_LIB_VARIANT=$v timeout -k 10 120 python bench.py --no-cpu-baseline --no-gather --steps 2000 --no-kernel-events |
    python -c "import json,sys; d=json.load(sys.stdin); print(round(d['value']/1e6,1), 'M agent-steps/s', d['ms_per_step'], 'ms/step')"
done
