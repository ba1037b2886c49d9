set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_sweep.sh cfg4 1 "" x_noscan x_nob x_noplan
bash tools/ab_sweep.sh cfg2 1 ""
