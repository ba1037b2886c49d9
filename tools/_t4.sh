set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_sweep.sh cfg3 2 "" probepk probeint1
bash tools/ab_sweep.sh cfg2 1 "" probepk probeint1
