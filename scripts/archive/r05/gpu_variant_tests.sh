#!/bin/bash
# Full GPU test suite against prebuilt library variants (default =
# lib/libhashnerf_amd.so); stops at the first failing variant or crash.
#   usage: scripts/gpu_variant_tests.sh TAG NAME ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out
mkdir -p $OUT
for V in "$@"; do
  L=hashnerf-pytorch_amd/build/$V.so
  [ "$V" = "default" ] && L=hashnerf-pytorch_amd/lib/libhashnerf_amd.so
  HN_LIB_PATH=$L timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread \
      > $OUT/vt_${TAG}_$V.log 2>&1
  RC=$?
  echo "variant $V pytest rc=$RC: $(tail -1 $OUT/vt_${TAG}_$V.log)"
  [ $RC -le 1 ] || exit $RC
done
