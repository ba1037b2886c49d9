"""Static world of the device path vs the REFERENCE's own outputs.

tests/golden/static_lanes{2,3}.npz hold, from the reference build: the
is_on_road / hits_yellow_line / LineMask::is_line predicates on the full
750x750 integer grid and on random real points, and the 160-point path,
intent and spawn heading of every (start, end) lane-point pair.
mev_world.h / mev_routes.h (compiled for the host, same code as the kernels
and the route-table builder) must reproduce all of them bit-for-bit."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

import native_build
from golden_replay import GOLDEN_DIR


@pytest.mark.parametrize("lanes", [2, 3])
def test_world_matches_reference(lanes):
    z = np.load(os.path.join(GOLDEN_DIR, f"static_lanes{lanes}.npz"))
    exe = native_build.build("world_dump")
    with tempfile.TemporaryDirectory() as td:
        pre = os.path.join(td, "w")
        z["pts"].astype(np.float32).tofile(pre + ".pts")
        subprocess.run([exe, str(lanes), pre], check=True)
        grid = np.fromfile(pre + ".grid", np.uint8).reshape(750, 750)
        paths = np.fromfile(pre + ".paths", np.float32).reshape(-1, 160, 2)
        intent = np.fromfile(pre + ".intent", np.int32)
        spawn = np.fromfile(pre + ".spawn", np.float32).reshape(-1, 3)
        ptsout = np.fromfile(pre + ".ptsout", np.uint8).reshape(-1, 2)
    assert not (grid & 8).any(), "integer and real-valued road predicates disagree"
    ref = z["grid"]
    for bit, name in ((1, "is_on_road"), (2, "hits_yellow_line"), (4, "LineMask::is_line")):
        bad = np.argwhere((grid & bit) != (ref & bit))
        assert len(bad) == 0, f"{name} differs at {bad[:5].tolist()}"
    np.testing.assert_array_equal(ptsout[:, 0], z["road"])
    np.testing.assert_array_equal(ptsout[:, 1], z["yellow"])
    assert paths.shape == z["paths"].shape
    assert np.array_equal(paths.view(np.uint32), z["paths"].view(np.uint32)), "route paths differ"
    np.testing.assert_array_equal(intent, z["intent"])
    assert np.array_equal(spawn.view(np.uint32), z["spawn"].view(np.uint32)), "spawn (x, y, heading) differ"
