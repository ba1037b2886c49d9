#!/bin/bash
# HBM traffic of k_step from two separate PMC passes (FETCH_SIZE, WRITE_SIZE) for
# library variants: bash tools/pmc_traffic.sh "" noxcd ...  -> gpurun_out/pmc_<v>_{fetch,write}
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  tag=${v:-product}
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/pmc_${tag}_$c
    MEV_LIB_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc $c -d gpurun_out/pmc_${tag}_$c -o run --output-format csv -- \
      python3 bench.py --no-kernel-events --no-cpu-baseline --no-gather --steps 200 > gpurun_out/pmc_${tag}_$c.log 2>&1
  done
  python tools/pmc_traffic.py gpurun_out/pmc_${tag}_FETCH_SIZE gpurun_out/pmc_${tag}_WRITE_SIZE --envs 4096 --agents 8 --rays 64 --out gpurun_out/pmc_traffic_${tag}.json | tail -12
done
