#!/bin/bash
# r03h: new defaults (B-split pipelining in the MLP backward, staged scatter
# records).  Full GPU tests, smoke, PMC passes -> traffic json used by the
# bench line, the default bench (CPU baseline included), kernel stats, then
# A/B of prebuilt variants (hashnerf-pytorch_amd/build/var_*.so).
set -o pipefail
TAG=r03h
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu_$TAG.log 2>&1
RC=$?; echo "pytest rc=$RC"; grep -E "passed|failed" $OUT/pytest_gpu_$TAG.log | tail -3
[ $RC -le 1 ] || exit $RC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || exit 2
timeout -k 10 600 bash scripts/gpu_pmc.sh $TAG > $OUT/pmc_$TAG.out 2>&1 || exit 7
cp $OUT/traffic_$TAG.json profiles/traffic_config2_procedural_p1000_binned.json
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit 3
cat $OUT/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o prof -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 || exit 5
python3 scripts/trace_tail_stats.py $OUT/prof_$TAG/prof_kernel_trace.csv 10 > $OUT/prof_$TAG/prof_kernel_stats_timed.csv
rm -f $OUT/prof_$TAG/prof_kernel_trace.csv
head -10 $OUT/prof_$TAG/prof_kernel_stats_timed.csv | cut -c1-110
for V in base var_vgprform var_wgsb0 var_wgsb0vf var_nostage base var_vgprform var_wgsb0 var_wgsb0vf var_nostage; do
  if [ $V = base ]; then L=hashnerf-pytorch_amd/lib/libhashnerf_amd.so; else L=hashnerf-pytorch_amd/build/$V.so; fi
  HN_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/ab_$V.json 2> $OUT/ab_$V.err || exit 6
  python -c "import json;d=json.load(open('$OUT/ab_$V.json'));print('$V', d['value'], d['ms_per_step'], d['kernels']['render_fwd_ms'], d['kernels']['render_bwd_ms'])"
done
echo "chain ok"
