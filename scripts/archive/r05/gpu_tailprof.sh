#!/bin/bash
# rocprofv3 kernel trace of a short default bench; per-kernel stats of the
# timed steps only (scripts/trace_tail_stats.py).   usage: scripts/gpu_tailprof.sh TAG
set -o pipefail
TAG=${1:-t}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o prof -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 || { echo "prof failed"; tail $OUT/prof_$TAG.log; exit 1; }
python3 scripts/trace_tail_stats.py $OUT/prof_$TAG/prof_kernel_trace.csv 10 > $OUT/prof_$TAG/prof_kernel_stats_timed.csv
rm -f $OUT/prof_$TAG/prof_kernel_trace.csv
python3 -c "
import csv,sys
for r in list(csv.DictReader(open('$OUT/prof_$TAG/prof_kernel_stats_timed.csv')))[:24]:
    print(f'{float(r[\"AverageNs\"])/1e3:9.2f} us  {r[\"Name\"][:90]}')"
