#!/bin/bash
# r03m: ABI 10 (ReLU masks in the feature cache).  GPU tests on the default
# build and on the stored-mask build (2-part recompute), A/B of the variants.
set -o pipefail
TAG=r03m
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu_$TAG.log 2>&1
RC=$?; echo "pytest rc=$RC"; grep -E "passed|failed" $OUT/pytest_gpu_$TAG.log | tail -3
[ $RC -le 1 ] || exit $RC
HN_LIB_PATH=hashnerf-pytorch_amd/build/var_smask.so timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf \
    --timeout 120 --timeout-method thread --ignore tests/test_psnr.py > $OUT/pytest_smask_$TAG.log 2>&1
RC=$?; echo "pytest smask rc=$RC"; grep -E "passed|failed|FAILED" $OUT/pytest_smask_$TAG.log | tail -6
[ $RC -le 1 ] || exit $RC
for V in base var_smask var_scroll10 var_smask_scroll base var_smask var_scroll10 var_smask_scroll; do
  if [ $V = base ]; then L=hashnerf-pytorch_amd/lib/libhashnerf_amd.so; else L=hashnerf-pytorch_amd/build/$V.so; fi
  HN_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/ab_$V.json 2> $OUT/ab_$V.err || exit 6
  python -c "import json;d=json.load(open('$OUT/ab_$V.json'));print('$V', d['value'], d['ms_per_step'], d['kernels']['render_fwd_ms'], d['kernels']['render_bwd_ms'])"
done
for V in var_smask var_scroll10; do
  HN_LIB_PATH=hashnerf-pytorch_amd/build/$V.so timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG}_$V -o prof -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_${TAG}_$V.log 2>&1 || exit 5
  python3 scripts/trace_tail_stats.py $OUT/prof_${TAG}_$V/prof_kernel_trace.csv 10 > $OUT/prof_${TAG}_$V/prof_kernel_stats_timed.csv
  rm -f $OUT/prof_${TAG}_$V/prof_kernel_trace.csv
  echo "== $V"; head -6 $OUT/prof_${TAG}_$V/prof_kernel_stats_timed.csv | cut -c1-110
done
echo "chain ok"
