#!/bin/bash
# r03j: GPU tests on the new defaults (MFMA VGPR form, no barrier after
# weight-gradient chunks), then A/B of prebuilt variants.
set -o pipefail
TAG=r03j
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu_$TAG.log 2>&1
RC=$?; echo "pytest rc=$RC"; grep -E "passed|failed" $OUT/pytest_gpu_$TAG.log | tail -3
[ $RC -le 1 ] || exit $RC
HN_LIB_PATH=hashnerf-pytorch_amd/build/var_maskmin.so timeout -k 10 300 python -u -m pytest tests/test_gpu_driver.py tests/test_gpu_scatter.py -m gpu -q -rf \
    --timeout 120 --timeout-method thread > $OUT/pytest_maskmin_$TAG.log 2>&1
RC=$?; echo "pytest maskmin rc=$RC"; grep -E "passed|failed" $OUT/pytest_maskmin_$TAG.log | tail -2
[ $RC -le 1 ] || exit $RC
for V in base var_maskmin var_swp2_3 var_swp4_5 var_wgsb1 base var_maskmin var_swp2_3 var_swp4_5 var_wgsb1; do
  if [ $V = base ]; then L=hashnerf-pytorch_amd/lib/libhashnerf_amd.so; else L=hashnerf-pytorch_amd/build/$V.so; fi
  HN_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/ab_$V.json 2> $OUT/ab_$V.err || exit 6
  python -c "import json;d=json.load(open('$OUT/ab_$V.json'));print('$V', d['value'], d['ms_per_step'], d['kernels']['render_fwd_ms'], d['kernels']['render_bwd_ms'])"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o prof -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 || exit 5
python3 scripts/trace_tail_stats.py $OUT/prof_$TAG/prof_kernel_trace.csv 10 > $OUT/prof_$TAG/prof_kernel_stats_timed.csv
rm -f $OUT/prof_$TAG/prof_kernel_trace.csv
head -6 $OUT/prof_$TAG/prof_kernel_stats_timed.csv | cut -c1-110
HN_LIB_PATH=hashnerf-pytorch_amd/build/var_tileprof.so timeout -k 10 300 python bench.py --steps 4 --warmup 2 --no-cpu-baseline \
    > $OUT/tileprof_$TAG.json 2> $OUT/tileprof_$TAG.err || exit 7
grep "hn_b1_" $OUT/tileprof_$TAG.err | tail -4
timeout -k 10 400 bash scripts/gpu_psnr_diag2.sh 3 || exit 8
echo "chain ok"
