#!/bin/bash
# GPU A/B: build, GPU parity tests, then one short bench per environment
# variant (e.g. HN_SCATTER=atomic).  Every GPU step has its own time limit
# and the chain stops at the first abort / crash / timeout.
#   usage: scripts/gpu_ab.sh TAG "VAR=VAL ..." ["VAR=VAL ..." ...]   ("-" = default env)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
python hashnerf-pytorch_amd/build.py > $OUT/build_$TAG.log 2>&1 || { echo "build failed"; tail $OUT/build_$TAG.log; exit 1; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread \
      > $OUT/pytest_gpu_$TAG.log 2>&1
  RC=$?
  echo "pytest rc=$RC"; tail -4 $OUT/pytest_gpu_$TAG.log
  [ $RC -le 1 ] || exit $RC
fi
i=0
for V in "$@"; do
  i=$((i+1))
  [ "$V" = "-" ] && V=""
  env $V timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline ${BENCH_ARGS} \
      > $OUT/bench_${TAG}_$i.json 2> $OUT/bench_${TAG}_$i.err
  RC=$?
  echo "variant $i [$V] rc=$RC"
  [ $RC -eq 0 ] || { tail -5 $OUT/bench_${TAG}_$i.err; exit $RC; }
  python -c "import json;d=json.load(open('$OUT/bench_${TAG}_$i.json'));print(d['value'], d['ms_per_step'], d['kernels'])"
done
