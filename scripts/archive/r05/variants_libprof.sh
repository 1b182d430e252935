#!/bin/bash
# Prebuilt library variants (hashnerf-pytorch_amd/build/NAME.so, "default" =
# lib/libhashnerf_amd.so): the scatter/owner GPU tests, a short bench and the
# per-kernel averages of the timed steps (rocprofv3 --kernel-trace) for each.
#   usage: scripts/variants_libprof.sh TAG NAME ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for V in "$@"; do
  i=$((i+1))
  L=hashnerf-pytorch_amd/build/$V.so
  [ "$V" = "default" ] && L=hashnerf-pytorch_amd/lib/libhashnerf_amd.so
  export HN_LIB_PATH=$L
  if [ -z "$SKIP_TESTS" ]; then
    timeout -k 10 300 python -u -m pytest tests/test_gpu_scatter.py -x -q --timeout 120 --timeout-method thread \
        > $OUT/vl_${TAG}_$i.pytest 2>&1 || { echo "variant $V tests failed"; tail -5 $OUT/vl_${TAG}_$i.pytest; exit 1; }
  fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $BENCH_ARGS \
      > $OUT/vl_${TAG}_$i.json 2> $OUT/vl_${TAG}_$i.err || { echo "variant $V bench failed"; tail -3 $OUT/vl_${TAG}_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/vl_${TAG}_$i.json'));print('$V', d['value'], d['ms_per_step'])"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/vl_${TAG}_$i -o p -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline $BENCH_ARGS > $OUT/vl_${TAG}_$i.log 2>&1 \
      || { echo "variant $V prof failed"; tail -3 $OUT/vl_${TAG}_$i.log; exit 1; }
  T=$(ls $OUT/vl_${TAG}_$i/*kernel_trace.csv $OUT/vl_${TAG}_$i/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 scripts/trace_tail_stats.py $T 10 > $OUT/vl_${TAG}_$i.stats.csv
  rm -f $T
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/vl_${TAG}_$i.stats.csv')):
    if float(r['AverageNs']) > 12000: print(f'   {float(r[\"AverageNs\"])/1e3:9.2f} us  {r[\"Name\"][:60]}')"
done
