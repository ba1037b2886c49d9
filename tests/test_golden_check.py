"""The committed golden vectors are what the reference produces today: tests/golden/gen_golden.py
--check regenerates every deterministic scenario from the reference compiled here
(oracle/build_ref.sh -> $MEV_REF_BUILD/libref_harness.so) into a temporary directory and
compares each array of each file with the committed one, byte for byte.  Traffic scenarios
with spawns are not regenerated: the reference draws them from an unseeded RNG
(TrafficFlow.cpp:278,324); their recorded spawns are replayed instead.

Runs where the reference harness has been built (the build container); skipped elsewhere
(the GPU box has no reference)."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import refharness  # noqa: E402  (test infrastructure)


@pytest.mark.skipif(not refharness.available(), reason="reference harness not built (no /root/reference here)")
def test_goldens_regenerate_identically():
    r = subprocess.run([sys.executable, os.path.join(HERE, "golden", "gen_golden.py"), "--check"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "0 file(s) differ" in r.stdout
