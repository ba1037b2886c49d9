set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python tools/env_latency.py 2>&1 | grep -v amdgpu
timeout -k 10 300 python -u -m pytest tests/test_dropin_gpu.py tests/test_capi_c_example.py tests/test_snapshot_reset_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
