"""mev_math.h (the device libm) is bit-identical to this image's glibc libm on
the simulator's argument ranges (strided sweeps; `devmath_check exhaustive`
runs every float — see DESIGN.md)."""
import subprocess

import native_build


def test_devmath_matches_glibc():
    exe = native_build.build("devmath_check")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "DEVMATH OK" in r.stdout
