#!/bin/bash
# r03q: bisect the render forward's rare nondeterminism (r03p: 1 of 8
# identical forwards gave one ray different colour-net results on points
# 16-31 of every tile, features identical): default vs 2 waves per SIMD vs
# no MFMA-VGPR-form, 12 repeats each; then the GPU tests.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for V in default var_w2 var_novgpr; do
  if [ $V = default ]; then unset HN_LIB_PATH; else export HN_LIB_PATH=hashnerf-pytorch_amd/build/$V.so; fi
  timeout -k 10 300 python -u scripts/diag_fwd_det.py 4096 12 > $OUT/diag_fwd_det_${V}_r03q.log 2>&1 || exit 2
  echo "== $V"; grep -v amdgpu.ids $OUT/diag_fwd_det_${V}_r03q.log
done
unset HN_LIB_PATH
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu_r03q.log 2>&1
RC=$?; echo "pytest rc=$RC"; grep -E "passed|failed" $OUT/pytest_gpu_r03q.log | tail -3
echo "chain ok"
