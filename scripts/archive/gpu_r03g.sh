#!/bin/bash
# r03g: color_net.2^T on split-bf16 products + compiler-only LDS ordering in
# the MLP backward tile.  Full GPU tests, A/B against the two previous forms
# (prebuilt var_*.so), kernel stats, PMC passes (traffic + MFMA busy), bench.
set -o pipefail
TAG=r03g
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu_$TAG.log 2>&1
RC=$?; echo "pytest rc=$RC"; grep -E "passed|failed" $OUT/pytest_gpu_$TAG.log | tail -3
[ $RC -le 1 ] || exit $RC
HN_LIB_PATH=hashnerf-pytorch_amd/build/var_scstage.so timeout -k 10 300 python -u -m pytest tests/test_gpu_scatter.py -m gpu -v -rf \
    --timeout 120 --timeout-method thread > $OUT/pytest_scstage_$TAG.log 2>&1
RC=$?; echo "pytest scstage rc=$RC"; grep -E "passed|failed" $OUT/pytest_scstage_$TAG.log | tail -3
[ $RC -le 1 ] || exit $RC
for V in base var_b4f32 var_ldsfence var_b1swp var_gemmswp var_bothswp var_scstage base var_b4f32 var_ldsfence var_b1swp var_gemmswp var_bothswp var_scstage; do
  if [ $V = base ]; then L=hashnerf-pytorch_amd/lib/libhashnerf_amd.so; else L=hashnerf-pytorch_amd/build/$V.so; fi
  HN_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/ab_$V.json 2> $OUT/ab_$V.err || exit 6
  python -c "import json;d=json.load(open('$OUT/ab_$V.json'));print('$V', d['value'], d['ms_per_step'], d['kernels']['render_fwd_ms'], d['kernels']['render_bwd_ms'])"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o prof -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 || exit 5
python3 scripts/trace_tail_stats.py $OUT/prof_$TAG/prof_kernel_trace.csv 10 > $OUT/prof_$TAG/prof_kernel_stats_timed.csv
rm -f $OUT/prof_$TAG/prof_kernel_trace.csv
head -10 $OUT/prof_$TAG/prof_kernel_stats_timed.csv | cut -c1-110
timeout -k 10 600 bash scripts/gpu_pmc.sh $TAG > $OUT/pmc_$TAG.out 2>&1 || exit 7
HN_LIB_PATH=hashnerf-pytorch_amd/build/var_scstage.so PMC_PASSES="FETCH_SIZE;WRITE_SIZE" timeout -k 10 300 \
    bash scripts/gpu_pmc.sh ${TAG}_scstage > $OUT/pmc_${TAG}_scstage.out 2>&1 || exit 8
grep -A3 "scatter_bins\|bin_reduce" $OUT/pmc_${TAG}_scstage.txt
grep -A12 "render_bwd_kernel\|render_fwd_kernel" $OUT/pmc_$TAG.txt | head -40
echo "chain ok"
