#!/bin/bash
# Diagnostic: kernel trace of a short bench run and the dispatch timeline of
# its last timed steps (scripts/trace_timeline.py).   usage: scripts/gpu_timeline.sh [bench args...]
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tl -o tl -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > $OUT/timeline_bench.log 2>&1 || { tail -3 $OUT/timeline_bench.log; exit 1; }
T=$(ls $OUT/tl/*kernel_trace.csv $OUT/tl/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/trace_timeline.py $T 2 | tee $OUT/timeline.txt
rm -f $T
