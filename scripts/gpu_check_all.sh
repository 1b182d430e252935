#!/bin/bash
# Full check of the tree on one GPU: GPU tests, smoke, the config-2 bench
# line (with CPU baseline), a rocprofv3 kernel-trace summary of the bench.
#   usage: scripts/gpu_check_all.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-chk}
K=${2:-}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 170 --timeout-method thread "${KA[@]}" > $O/pytest_gpu.log 2>&1; RC=$?
tail -3 $O/pytest_gpu.log; [ $RC -eq 0 ] || exit $RC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python bench.py > $O/bench_full.json 2> $O/bench_full.err || { tail -5 $O/bench_full.err; exit 1; }
cut -c1-300 $O/bench_full.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
F=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_tail_stats.py $F 20 > $O/kernel_stats_$TAG.csv
S=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $S $O/rocprof_kernel_stats_$TAG.csv; rm -rf $O/prof
grep -o '"launch_ms": [0-9.]*\|"render_fwd_ms": [0-9.]*' $O/prof.log | head -3
cut -d, -f1,2,4 $O/kernel_stats_$TAG.csv | head -8
