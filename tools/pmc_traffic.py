"""Per-launch HBM traffic of the step kernels from rocprofv3 PMC passes.

Usage (on the GPU box, two separate passes — FETCH_SIZE and WRITE_SIZE do not
fit one TCC pass on gfx950):
    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py ...
    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --envs 4096 --agents 8 --rays 64

Writes profiles/pmc_traffic.json: per kernel, the mean FETCH_SIZE and
WRITE_SIZE per launch (rocprofv3 reports KB), the gfx950 correction of
MI355X_MICROARCH.md §HBM (FETCH_SIZE counts half the bytes of wide coalesced
reads: doubled), and hbm_bytes_per_launch = 2*FETCH + WRITE in bytes.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def _read(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise FileNotFoundError(f"no counter_collection.csv under {d}")
    per = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                name = row["Kernel_Name"]
                if "mev::" not in name:
                    continue            # the library's kernels only (not torch's input generation)
                for short in ("k_step", "k_lidar", "k_cars", "k_reset", "k_restore"):
                    if short in name:
                        name = short + name[name.find(short) + len(short):].split("(")[0]
                        break
                per[name].append(float(row["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--envs", type=int, required=True)
    ap.add_argument("--agents", type=int, required=True)
    ap.add_argument("--rays", type=int, required=True)
    ap.add_argument("--skip", type=int, default=10, help="launches per kernel to skip (warm-up)")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    fetch = _read(a.fetch_dir, "FETCH_SIZE")
    write = _read(a.write_dir, "WRITE_SIZE")
    res = {"envs": a.envs, "agents": a.agents, "rays": a.rays,
           "note": "FETCH_SIZE/WRITE_SIZE are KB per dispatch (rocprofv3); hbm_bytes_per_launch = "
                   "(2*FETCH_SIZE + WRITE_SIZE) * 1024, the x2 being the gfx950 FETCH_SIZE correction "
                   "(MI355X_MICROARCH.md, HBM section)"}
    for k in sorted(set(fetch) & set(write)):
        f = fetch[k][a.skip:] or fetch[k]
        w = write[k][a.skip:] or write[k]
        fk, wk = sum(f) / len(f), sum(w) / len(w)
        res[k.split("<")[0] if k.split("<")[0] not in res else k] = {
            "kernel": k, "launches": len(f), "fetch_size_kb": round(fk, 3), "write_size_kb": round(wk, 3),
            "hbm_bytes_per_launch": round((2 * fk + wk) * 1024.0, 1)}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
