set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/t3; mkdir -p $O
rm -rf $O/ic1 $O/ic2
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d $O/ic1 -o run --output-format csv -- python3 bench.py --no-kernel-events --no-cpu-baseline --no-gather --steps 200 > $O/ic1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQC_TC_INST_REQ SQ_WAVES SQ_WAIT_INST_ANY -d $O/ic2 -o run --output-format csv -- python3 bench.py --no-kernel-events --no-cpu-baseline --no-gather --steps 200 > $O/ic2.log 2>&1
python tools/pmc_sq.py $O/ic1 > $O/ic1.txt; python tools/pmc_sq.py $O/ic2 > $O/ic2.txt
cat $O/ic1.txt $O/ic2.txt
