"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean per dispatch and
per wave).  python tools/pmc_sq.py <dir> [--skip N]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 5
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"]
                if "mev::" not in name:
                    continue
                name = name.split("(")[0].replace("void ", "")
                vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in sorted(vals.items()):
        waves = cs.get("SQ_WAVES")
        wv = (sum(waves[skip:]) / max(1, len(waves[skip:]))) if waves else None
        print(k)
        for c, v in sorted(cs.items()):
            v = v[skip:] or v
            m = sum(v) / len(v)
            per = f"  per wave {m / wv:12.1f}" if wv and c != "SQ_WAVES" else ""
            print(f"  {c:24s} {m:16.1f}{per}")


if __name__ == "__main__":
    main()
