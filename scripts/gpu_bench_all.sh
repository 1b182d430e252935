#!/bin/bash
# Bench lines of configs 2 (default), 3, 4 and 5 on one GPU, each with its
# CPU baseline, plus a rocprof kernel summary of configs 3 and 5.
#   usage: scripts/gpu_bench_all.sh TAG [configs...]
set -o pipefail
TAG=${1:-b}
shift
CFGS=${@:-2 3 4 5}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for C in $CFGS; do
  timeout -k 10 600 python bench.py --config $C > $O/bench_config${C}.json 2> $O/bench_config${C}.err \
      || { tail -5 $O/bench_config${C}.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_config${C}.json'));print('config $C', d['value'], d['ms_per_step'], d['kernels']['render_fwd_ms'], d['kernels']['render_bwd_ms'], d.get('cpu_baseline',{}).get('value'))"
done
if [ -n "$PROF" ]; then
  for C in $PROF; do
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof$C -o prof -- python3 bench.py --config $C \
        --steps 10 --warmup 3 --no-cpu-baseline > $O/prof$C.log 2>&1 || { tail -5 $O/prof$C.log; exit 1; }
    F=$(find $O/prof$C -name "*kernel_trace.csv" | head -1)
    python3 scripts/trace_tail_stats.py $F 20 > $O/kernel_stats_config${C}.csv && rm -rf $O/prof$C
    cut -d, -f1,2,4 $O/kernel_stats_config${C}.csv | head -6 | sed "s/^/config $C /"
  done
fi
