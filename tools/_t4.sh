set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_sweep.sh cfg4 2 "" trafprio2 trafprio3
