"""The driver's short bench run (bench.py --gpus 1 --steps K --warmup W) under
rocprofv3 --kernel-trace: per-dispatch durations and inter-dispatch gaps of the
metric phase's K timed k_step launches, beside the bench line's own numbers.

    rocprofv3 --kernel-trace -d OUT -o run -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
    python tools/short_run_trace.py OUT/run_kernel_trace.csv --steps 20 --warmup 5 [--line bench_line.json]

Phase 1 of bench.py (the metric) is: the clock settle's steps, k_reset, W warm-up
and K timed steps; phase 2 (the gather) starts with the next k_reset.  So the timed
launches are the K k_step dispatches right before the second k_reset after the
settle."""
import argparse
import csv
import json

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--line", default=None, help="the bench's JSON line (file) to compare with")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    kind = []
    for r in rows:
        n = r["Kernel_Name"]
        kind.append("step" if "k_step" in n else ("reset" if "k_reset" in n else "other"))
    resets = [i for i, k in enumerate(kind) if k == "reset"]
    # the settle ends with a reset; the metric phase's W + K steps follow it
    assert len(resets) >= 2, "expected the settle's reset and the gather phase's reset"
    r0 = resets[-2] if len(resets) >= 2 else resets[0]
    steps = [i for i in range(r0 + 1, len(rows)) if kind[i] == "step"][: a.warmup + a.steps]
    timed = steps[a.warmup:]
    assert len(timed) == a.steps, (len(timed), a.steps)
    st = np.array([int(rows[i]["Start_Timestamp"]) for i in timed], np.int64)
    en = np.array([int(rows[i]["End_Timestamp"]) for i in timed], np.int64)
    dur = (en - st) / 1e3
    gaps = (st[1:] - en[:-1]) / 1e3
    settle = [i for i in range(resets[-2] if len(resets) >= 2 else 0) if kind[i] == "step"]
    sd = np.array([(int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3 for i in settle[-1000:]])
    out = {
        "timed_dispatches": a.steps,
        "kernel_us_mean": round(float(dur.mean()), 3), "kernel_us_min": round(float(dur.min()), 3),
        "kernel_us_max": round(float(dur.max()), 3),
        "kernel_us_each": [round(float(x), 2) for x in dur],
        "gap_us_mean": round(float(gaps.mean()), 3), "gap_us_max": round(float(gaps.max()), 3),
        "first_start_to_last_end_us_per_step": round(float((en[-1] - st[0]) / 1e3 / a.steps), 3),
        "settle_last_1000_kernel_us_mean": round(float(sd.mean()), 3) if len(sd) else None,
        "kernel_name": rows[timed[0]]["Kernel_Name"],
    }
    if a.line:
        d = json.loads(open(a.line).read().strip().splitlines()[-1])
        out["bench_ms_per_step"] = d["ms_per_step"]
        out["bench_stream_kernel_ms"] = d["roofline"]["kernel_ms"]
        out["bench_value"] = d["value"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
