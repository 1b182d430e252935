#!/bin/bash
# A/B of prebuilt variant libraries (hashnerf-pytorch_amd/build/<name>.so, built
# on the CPU side with build.build_variant), interleaved REPS times on one box:
# short bench lines (forward/backward launch times from HIP events), then one
# rocprofv3 kernel trace per variant (the last 10 timed steps' kernel stats).
#   usage: REPS=2 scripts/gpu_lib_ab.sh TAG var_a var_b ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 ${REPS:-2}); do
  for V in "$@"; do
    HN_LIB_PATH=hashnerf-pytorch_amd/build/$V.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 \
        --no-cpu-baseline $BENCH_ARGS > $OUT/${V}_$r.json 2> $OUT/${V}_$r.err || { tail -5 $OUT/${V}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/${V}_$r.json'));print('$V', $r, d['value'], d['ms_per_step'], d['kernels']['render_fwd_ms'], d['kernels']['render_bwd_ms'])"
  done
done
if [ -n "$PROF" ]; then
  for V in "$@"; do
    HN_LIB_PATH=hashnerf-pytorch_amd/build/$V.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
        -d $OUT/prof_$V -o prof -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline $BENCH_ARGS \
        > $OUT/prof_$V.log 2>&1 || { tail -5 $OUT/prof_$V.log; exit 1; }
    F=$(find $OUT/prof_$V -name "*kernel_trace.csv" | head -1)
    python3 scripts/trace_tail_stats.py $F 10 > $OUT/kernel_stats_$V.csv && rm -rf $OUT/prof_$V
    grep -h "render_fwd_kernel\|render_bwd_kernel\|scatter_bins\|bin_reduce" $OUT/kernel_stats_$V.csv | cut -d, -f1,2,4 | sed "s/^/$V /"
  done
fi
