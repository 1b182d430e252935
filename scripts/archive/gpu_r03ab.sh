#!/bin/bash
# r03ab: two scheduling-only variants (bitwise-identical results) A/B'd
# against the final defaults on one box: HN_GEMM_PF=0 (forward fragments
# loaded at use), HN_B1_LANE_OPAQUE=0 (the MLP backward may keep its LDS image
# addresses across tiles); then each variant's GPU tests.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for R in 1 2; do
  for V in base var_gemmpf0 var_laneopq0; do
    if [ $V = base ]; then unset HN_LIB_PATH; else export HN_LIB_PATH=hashnerf-pytorch_amd/build/$V.so; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/ab_${V}_r03ab_$R.json 2> $OUT/ab_${V}_r03ab_$R.err || exit 8
    python -c "import json;d=json.load(open('$OUT/ab_${V}_r03ab_$R.json'));print('$V', d['value'], d['ms_per_step'], d['kernels']['render_fwd_ms'], d['kernels']['render_bwd_ms'])"
  done
done
for V in var_gemmpf0 var_laneopq0; do
  export HN_LIB_PATH=hashnerf-pytorch_amd/build/$V.so
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $OUT/pytest_gpu_${V}_r03ab.log 2>&1
  RC=$?; echo "$V pytest rc=$RC: $(tail -1 $OUT/pytest_gpu_${V}_r03ab.log)"
  [ $RC -le 1 ] || exit $RC
done
echo "chain ok"
