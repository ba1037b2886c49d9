set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in stamps stampsx stampsy; do
MEV_LIB_VARIANT=$v timeout -k 10 120 python tools/phase_profile.py --envs 256 --agents 1 --step-kernel 2 2>&1 | grep -v amdgpu.ids
done
MEV_LIB_VARIANT=stampsr timeout -k 10 120 python tools/simd_balance.py --envs 4096 2>&1 | grep -v amdgpu.ids
