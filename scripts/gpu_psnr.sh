#!/bin/bash
# One paired PSNR@5k run (HIP trainer vs reference path) at seed $1.
#   usage: scripts/gpu_psnr.sh SEED TAG
set -o pipefail
SEED=${1:-0}
TAG=${2:-r01}
OUT=gpurun_out
mkdir -p $OUT
HN_PSNR_SEED=$SEED HN_PSNR_ITERS=5000 HN_PSNR_EVERY=100 HN_PSNR_RES=200 HN_PSNR_NTRAIN=100 \
HN_PSNR_OUT=$OUT/psnr_5k_${TAG}_seed$SEED.json \
    timeout -k 10 1000 python -u -m pytest tests/test_psnr.py -v -s --timeout 980 --timeout-method thread \
    > $OUT/psnr_5k_${TAG}_seed$SEED.log 2>&1
RC=$?
grep "^{" $OUT/psnr_5k_${TAG}_seed$SEED.log | tail -1
exit $RC
