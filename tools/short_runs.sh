#!/bin/bash
# round 6: the driver's exact short command (3x) + a rocprofv3 kernel trace of it; the config-5 line
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/r6b_short_$i.json 2> $O/r6b_short_$i.err
  python -c "import json; d=json.load(open('$O/r6b_short_$i.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
rm -rf $O/r6b_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r6b_trace -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/r6b_trace_line.json 2> $O/r6b_trace.err
f=$(find $O/r6b_trace -name '*kernel_trace.csv' | head -1)
python tools/short_run_trace.py $f --steps 20 --warmup 5 --line $O/r6b_trace_line.json > $O/r6b_trace_summary.json
cat $O/r6b_trace_summary.json | head -30
timeout -k 10 300 python bench.py --config 5 > $O/r6b_cfg5.json 2> $O/r6b_cfg5.err
cat $O/r6b_cfg5.json | cut -c1-600
