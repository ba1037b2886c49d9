set -e
cd $GRAFT_REPO_ROOT
for v in stampsx stampsy stamps; do
  for e in 4096 1024; do
    echo "== $v envs=$e"
    MEV_LIB_VARIANT=$v timeout -k 10 120 python tools/phase_profile.py --envs $e --step-kernel 2 --steps 100 2>&1 | grep -v amdgpu.ids
  done
done
