set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof2; mkdir -p $O
MEV_LIB_VARIANT=stamps timeout -k 10 200 python tools/npc_profile.py > $O/npc.txt 2>&1
MEV_LIB_VARIANT=stampsn timeout -k 10 200 python tools/npc_profile.py --parts > $O/npc_parts.txt 2>&1
cat $O/*.txt | grep -v amdgpu.ids
