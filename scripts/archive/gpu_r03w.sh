#!/bin/bash
# r03w: why the r03u PSNR runs printed nothing in 12 minutes -- one short run
# (300 iterations, an evaluation every 50) with a pytest timeout that dumps
# the stack where it hangs.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
HN_PSNR_SEED=0 HN_PSNR_ITERS=300 HN_PSNR_EVERY=50 HN_PSNR_RES=200 HN_PSNR_NTRAIN=100 HN_PSNR_NTEST=8 \
  timeout -k 10 200 python -u -m pytest tests/test_psnr.py -q -s -p no:cacheprovider --timeout 150 --timeout-method thread \
  > $OUT/psnr_short_r03w.log 2>&1
echo "rc=$?"; tail -60 $OUT/psnr_short_r03w.log
