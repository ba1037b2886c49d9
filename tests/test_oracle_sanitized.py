"""The C restatement under AddressSanitizer + UndefinedBehaviorSanitizer
(SURVEY.md §5): oracle/sanitize_replay.c (marl_oracle.c as one translation
unit, gcc -fsanitize=address,undefined) replays golden scenarios recorded from
the reference; any sanitizer report fails the run, and the outputs must still
equal the golden outputs bit for bit (the sanitized build changes no result)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

import golden_replay as G
import oracle_replay as R

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
EXE = os.path.join(ORACLE, "_build", "sanitize_replay")

# a spread of the golden set: single agent, team/8 agents, ties, traffic with spawns, NPC fleets, 128 beams,
# custom reward + dt, 2 lanes, truncation, unclipped actions
SCENARIOS = ["cfg1_r16_random", "cfg3_team_random_s0", "n16_r96_ties", "traffic_d20", "inject_npc_k9",
             "cfg5_r128_team", "dt_1_30_custom_reward", "lanes2_policy", "truncate_50", "unclipped_x3",
             "set_state_72_team"]


@pytest.fixture(scope="module")
def exe():
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    src = os.path.join(ORACLE, "sanitize_replay.c")
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < max(os.path.getmtime(src),
                                                               os.path.getmtime(os.path.join(ORACLE, "marl_oracle.c"))):
        # per-process temporary + atomic rename: pytest-xdist workers may build it at the same time
        tmp = f"{EXE}.{os.getpid()}.tmp"
        subprocess.run(["gcc", "-O1", "-g", "-std=c11", "-ffp-contract=off", "-fno-omit-frame-pointer",
                        "-fsanitize=address,undefined", "-fno-sanitize-recover=all", src, "-o", tmp, "-lm"],
                       check=True, capture_output=True)
        os.replace(tmp, EXE)
    return EXE


def _write_input(path, name):
    d = G.load(name)
    meta = d["meta"]
    L = int(meta["num_lanes"])
    n = int(meta["n_agents"])
    rays = int(meta["rays"])
    obs_dim = 127 if rays <= 96 else 31 + rays
    env = R.make_oracle(meta)  # only for route ids (s * P + t)
    tr = [env.route_id(G.point_index(s, L), G.point_index(e, L)) for s, e in meta["traffic_routes"]]
    ego_routes = [env.route_id(G.point_index(s, L), G.point_index(e, L)) for s, e in meta["ego_routes"]]
    egos = R.state_from_records(d["init_ego_f"], d["init_ego_i"], ego_routes)
    k = len(d["init_npc_f"])
    npcs = R.state_from_records(d["init_npc_f"], d["init_npc_i"], [tr[r] for r in d["init_npc_i"][:, 3]]) if k \
        else R.O.new_cars(0)
    steps = int(meta["steps"])
    hdr = np.array([L, n, rays, obs_dim, int(bool(meta["use_team"])), int(bool(meta["respawn"])),
                    int(meta["max_steps"]), int(bool(meta["traffic"])), 64, steps, len(tr), k,
                    int(meta.get("init_step", 0))], np.int32)
    fh = np.concatenate([[np.float32(meta["density"]), np.float32(meta["dt"])],
                         np.asarray(meta["reward"], np.float32)]).astype(np.float32)
    spawned = np.asarray(d["spawned"], np.int32) if meta["traffic"] else np.full(steps, -1, np.int32)
    with open(path, "wb") as f:
        for a in (hdr, fh, np.asarray(tr, np.int32), egos, npcs,
                  np.ascontiguousarray(d["actions"][:steps], np.float32), spawned[:steps]):
            f.write(np.ascontiguousarray(a).tobytes())
    return d, n, obs_dim, steps


@pytest.mark.parametrize("name", SCENARIOS)
def test_sanitized_oracle_replays_golden(exe, name, tmp_path):
    inp, outp = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
    d, n, D, steps = _write_input(inp, name)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, inp, outp], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    rec = np.dtype([("obs", np.float32, (n, D)), ("rew", np.float32, (n,)), ("done", np.uint8, (n,)),
                    ("status", np.uint8, (n,)), ("flags", np.int32, (4,))])
    raw = open(outp, "rb").read()
    per = rec.itemsize
    assert len(raw) == per * steps
    for t in range(steps):
        o = np.frombuffer(raw[t * per:(t + 1) * per], rec)[0]
        assert G.bits_equal(o["obs"][:, :127], d["obs"][t]), (name, t, "obs")
        assert G.bits_equal(o["rew"], d["rew"][t]), (name, t, "reward")
        assert np.array_equal(o["status"], d["status"][t]) and np.array_equal(o["done"], d["done"][t]), (name, t)
        assert [int(x) for x in o["flags"]] == [int(x) for x in d["flags"][t]], (name, t, "flags")
