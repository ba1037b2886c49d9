"""Write profiles/valu_counters.json from a rocprofv3 --pmc pass over bench.py
(SQ_INSTS_VALU, SQ_INSTS_SALU, SQ_INSTS_LDS, SQ_WAVES, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES...):
mean per k_step dispatch (the first --skip dispatches dropped).  bench.py's
roofline.valu divides SQ_INSTS_VALU per launch by the live kernel time.
    python tools/valu_counters.py <pmc dir> [--envs 4096 --agents 8 --rays 64 --skip 5] [--out file]"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--rays", type=int, default=64)
    ap.add_argument("--skip", type=int, default=5)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "valu_counters.json"))
    args = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(args.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"]
                if "mev::k_step" not in name:
                    continue
                vals["k_step"][row["Counter_Name"]].append(float(row["Counter_Value"]))
                vals["k_step"]["_name"] = name.split("(")[0].replace("void ", "")
    out = {"envs": args.envs, "agents": args.agents, "rays": args.rays,
           "note": "rocprofv3 --pmc pass of bench.py (config 3); mean per k_step dispatch; SQ_WAVE_CYCLES and the "
                   "SQ_WAIT/ACTIVE counters count quad-cycles (MI355X_MICROARCH.md)"}
    for k, cs in vals.items():
        d = {"kernel": cs.pop("_name")}
        waves = cs.get("SQ_WAVES", [])
        nw = sum(waves[args.skip:]) / max(1, len(waves[args.skip:])) if waves else None
        for c, v in sorted(cs.items()):
            v = v[args.skip:] or v
            m = sum(v) / len(v)
            d[c + "_per_launch"] = round(m, 1)
            if nw and c != "SQ_WAVES":
                d[c + "_per_wave"] = round(m / nw, 1)
        d["launches"] = len(waves)
        out[k] = d
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
