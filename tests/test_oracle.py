"""Pin the C restatement (oracle/marl_oracle.c) to the REAL reference: every
golden scenario (tests/golden/*.npz, generated from the reference build) must
replay bit-exactly.  Only then is the oracle used as a checker for the device
path on inputs the golden set does not cover (tests/test_gpu_vs_oracle.py)."""
import numpy as np
import pytest

import golden_replay as G
import oracle_replay as R


@pytest.mark.parametrize("name", G.scenario_names())
def test_oracle_matches_reference(name):
    errs = R.replay(name)
    assert not errs, f"{name}: {errs[:5]}"


@pytest.mark.parametrize("lanes", [2, 3])
def test_oracle_routes_match_reference(lanes):
    import os
    z = np.load(os.path.join(G.GOLDEN_DIR, f"static_lanes{lanes}.npz"))
    env = R.O.OracleEnv(num_lanes=lanes)
    P = env.P
    for r in range(P * P):
        path, intent = env.route_path(r)
        assert G.bits_equal(path, z["paths"][r]), f"route {r}"
        assert intent == z["intent"][r]
