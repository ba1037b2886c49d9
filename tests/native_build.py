"""Build helpers for the host-side native checks (tests/native/*.cpp)."""
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "marl-traffic-intersection_amd", "csrc")
OUT = os.path.join(tempfile.gettempdir(), "mev_native_tests")


def build(name: str, c_sources=()) -> str:
    """tests/native/<name>.cpp, plus plain-C sources (compiled as C and linked in)."""
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(HERE, "native", name + ".cpp")
    exe = os.path.join(OUT, name)
    deps = [src] + list(c_sources) + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    if os.path.exists(exe) and all(os.path.getmtime(d) <= os.path.getmtime(exe) for d in deps):
        return exe
    objs = []
    for c in c_sources:  # the same flags as oracle.build()
        o = os.path.join(OUT, os.path.basename(c) + ".o")
        subprocess.run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-c", c, "-o", o], check=True,
                       capture_output=True)
        objs.append(o)
    # same rounding discipline as the device build: no contraction, plain x86-64
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", "-I", CSRC, src, *objs, "-o", exe,
                    "-lm"], check=True, capture_output=True)
    return exe
