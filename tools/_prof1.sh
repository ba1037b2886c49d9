set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof1; mkdir -p $O
for cfg in "4096 8" "1024 8" "4096 1" "1024 1"; do set -- $cfg
  MEV_LIB_VARIANT=stampsr timeout -k 10 120 python tools/simd_balance.py --envs $1 --agents $2 > $O/bal_$1_$2.txt 2>&1
  for v in stamps stampsx stampsy; do
    MEV_LIB_VARIANT=$v timeout -k 10 120 python tools/phase_profile.py --envs $1 --agents $2 --step-kernel 2 --steps 100 > $O/${v}_$1_$2.txt 2>&1
  done
done
cat $O/*.txt | grep -v amdgpu.ids
