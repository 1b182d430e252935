#!/bin/bash
# A/B with per-kernel stats: for each environment variant, a short bench and a
# rocprofv3 kernel trace of the timed steps (scripts/gpu_tailprof.sh).
#   usage: scripts/gpu_ab_prof.sh TAG "VAR=VAL ..." ...   ("-" = default env)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
python hashnerf-pytorch_amd/build.py > $OUT/build_$TAG.log 2>&1 || { echo "build failed"; tail $OUT/build_$TAG.log; exit 1; }
i=0
for V in "$@"; do
  i=$((i+1))
  [ "$V" = "-" ] && V=""
  env $V timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline ${BENCH_ARGS} \
      > $OUT/bench_${TAG}_$i.json 2> $OUT/bench_${TAG}_$i.err || { echo "bench $i failed"; tail -5 $OUT/bench_${TAG}_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_${TAG}_$i.json'));print('variant $i [$V]', d['value'], d['ms_per_step'], d['kernels'])"
  env $V bash scripts/gpu_tailprof.sh ${TAG}_$i > $OUT/tail_${TAG}_$i.txt || exit 1
  head -7 $OUT/tail_${TAG}_$i.txt
done
