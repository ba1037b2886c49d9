"""The C ABI used from plain C (examples/capi_rollout.c): it compiles and links
against include/marlenv.h + libmarlenv_hip.so with gcc (CPU), and on the GPU
its rollout matches the same rollout through the Python binding."""
import os
import subprocess

import numpy as np
import pytest

import pkgload

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "examples", "capi_rollout.c")
PKG = os.path.join(ROOT, "marl-traffic-intersection_amd")


def _build(tmp_path):
    pkgload.load().load_library()  # builds libmarlenv_hip.so if hipcc is here
    exe = str(tmp_path / "capi_rollout")
    subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"), SRC,
                    "-L", PKG, "-lmarlenv_hip", f"-Wl,-rpath,{PKG}", "-o", exe], check=True)
    return exe


def test_c_example_compiles_and_links(tmp_path):
    exe = _build(tmp_path)
    assert os.access(exe, os.X_OK)


def _xorshift_actions(n, steps):
    xs = 12345
    out = np.zeros((steps, n), np.float32)
    for t in range(steps):
        for i in range(n):
            xs ^= (xs << 13) & 0xFFFFFFFF
            xs ^= xs >> 17
            xs ^= (xs << 5) & 0xFFFFFFFF
            out[t, i] = np.float32(np.float32(xs >> 8) * np.float32(2.0 / 16777216.0)) - np.float32(1.0)
    return out


@pytest.mark.gpu
def test_c_example_matches_python_binding(tmp_path):
    exe = _build(tmp_path)
    E, N, R, T = 8, 8, 64, 6
    r = subprocess.run([exe, str(E), str(N), str(R), str(T)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = [ln.split() for ln in r.stdout.strip().splitlines()]
    assert len(lines) == T
    mev = pkgload.load()
    h = mev.Handle(num_envs=E, num_agents=N, lidar_rays=R, use_team_reward=1)
    acts = _xorshift_actions(E * N * 2, T).reshape(T, E, N, 2)
    for t in range(T):
        o = h.step(acts[t], 1.0 / 60.0, auto_reset=True)
        osum = float(np.sum(o["obs"].astype(np.float64)))
        rsum = float(np.sum(o["reward"].astype(np.float64)))
        assert abs(osum - float(lines[t][3])) <= 1e-5 * max(1.0, abs(osum)), t
        assert abs(rsum - float(lines[t][5])) <= 1e-5 * max(1.0, abs(rsum)), t
        assert int((o["status"] >= 3).sum()) == int(lines[t][7]), t
    h.close()
