#!/bin/bash
# r03x: three short PSNR runs (300 iterations) at once on the one GPU, each
# with a pytest timeout that dumps its stack: does concurrency hang them?
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
PIDS=()
for S in 0 1 2; do
  HN_PSNR_SEED=$S HN_PSNR_ITERS=300 HN_PSNR_EVERY=50 HN_PSNR_RES=200 HN_PSNR_NTRAIN=100 HN_PSNR_NTEST=8 OMP_NUM_THREADS=1 \
    timeout -k 10 220 python -u -m pytest tests/test_psnr.py -q -s -p no:cacheprovider --timeout 180 --timeout-method thread \
    > $OUT/psnr_par_r03x_$S.log 2>&1 &
  PIDS+=($!)
done
( for i in 1 2 3 4; do sleep 50; echo "[$(date +%T)] $(tail -qn1 $OUT/psnr_par_r03x_0.log | cut -c1-80)"; done ) &
for P in "${PIDS[@]}"; do wait $P; echo "rc=$?"; done
for S in 0 1 2; do echo "== $S"; grep -v amdgpu.ids $OUT/psnr_par_r03x_$S.log | tail -40; done
