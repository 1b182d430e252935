#!/bin/bash
# A/B of variant libraries: REPS interleaved bench lines + one kernel profile each.
#   usage: REPS=2 scripts/gpu_ab_var.sh TAG var_a var_b ...
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in $(seq 1 ${REPS:-2}); do
  for V in "$@"; do
    HN_LIB_PATH=hashnerf-pytorch_amd/build/$V.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 $BENCH_ARGS \
        > $O/${V}_$r.json 2> $O/${V}_$r.err || { tail -5 $O/${V}_$r.err; exit 1; }
    echo "$V $r $(grep -o '"ms_per_step": [0-9.]*' $O/${V}_$r.json)"
  done
done
for V in "$@"; do
  HN_LIB_PATH=hashnerf-pytorch_amd/build/$V.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
      -d $O/prof_$V -o prof -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline $BENCH_ARGS \
      > $O/prof_$V.log 2>&1 || { tail -5 $O/prof_$V.log; exit 1; }
  F=$(find $O/prof_$V -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_tail_stats.py $F 10 > $O/kernel_stats_$V.csv && rm -rf $O/prof_$V
  cut -d, -f1,2,4 $O/kernel_stats_$V.csv | grep "hn::\|radam\|pack" | cut -c1-90 | sed "s/^/$V /"
done
