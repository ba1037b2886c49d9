set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MEV_LIB_VARIANT=stampsn timeout -k 10 200 python tools/npc_profile.py --parts 2>&1 | grep -v amdgpu
