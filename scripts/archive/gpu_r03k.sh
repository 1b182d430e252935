#!/bin/bash
# r03k: GPU tests, A/B (one b1_tile copy vs four; next-unit feature prefetch),
# then paired PSNR@5k seeds run one after the other (several processes on the
# one GPU slow each other down >5x on these boxes: gpurun_out/psnr_diag).
#   usage: scripts/gpu_r03k.sh SEED...
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TEST_RC=0
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread \
      > $OUT/pytest_gpu_r03k.log 2>&1
  RC=$?; echo "pytest rc=$RC"; grep -E "passed|failed" $OUT/pytest_gpu_r03k.log | tail -3
  [ $RC -le 1 ] || exit $RC
  TEST_RC=$RC
fi
for V in ${AB_VARIANTS:-base var_fourcopy var_prefetch base var_fourcopy var_prefetch}; do
  if [ $V = base ]; then L=hashnerf-pytorch_amd/lib/libhashnerf_amd.so; else L=hashnerf-pytorch_amd/build/$V.so; fi
  HN_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/ab_$V.json 2> $OUT/ab_$V.err || exit 6
  python -c "import json;d=json.load(open('$OUT/ab_$V.json'));print('$V', d['value'], d['ms_per_step'], d['kernels']['render_fwd_ms'], d['kernels']['render_bwd_ms'])"
done
[ $TEST_RC -eq 0 ] || { echo "tests failed: no PSNR runs"; exit 1; }
[ $# -gt 0 ] && HN_PSNR_PAR=1 HN_PSNR_TIMEOUT=560 bash scripts/gpu_psnr_multi.sh r03k "$@"
