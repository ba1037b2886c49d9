"""The neighbour order of get_observations is std::sort's (cpp/IntersectionEnv.cpp:490),
which is not stable above 16 candidates.  Both restatements -- the device's
(csrc/mev_nsort.h, host-compiled) and the oracle's (oracle/marl_oracle.c) -- are compared
with this image's libstdc++ std::sort itself on 32 000 arrays: exact ties, sorted /
reversed / constant inputs and McIlroy's adversary (which drives the sort into its
heapsort fallback)."""
import os
import subprocess

import native_build


def test_neighbour_sort_matches_libstdcxx():
    exe = native_build.build("nsort_check", [os.path.join(native_build.ROOT, "oracle", "marl_oracle.c")])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "NSORT OK" in r.stdout
