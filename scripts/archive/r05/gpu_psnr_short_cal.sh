#!/bin/bash
# Calibration of the short PSNR gate: paired 400-iteration runs (the default
# test) over SEEDS, curve every 25 iterations, optionally with the HIP side's
# learning rate scaled (HN_PSNR_LR_SCALE: a deliberate regression).
#   usage: SEEDS="0 1 2" LRS="1 0.7" scripts/gpu_psnr_short_cal.sh TAG
set -o pipefail
TAG=$1
OUT=gpurun_out/psnr_short_$TAG; mkdir -p $OUT
for LR in ${LRS:-1}; do
  for S in ${SEEDS:-0 1 2 3}; do
    HN_PSNR_SEED=$S HN_PSNR_EVERY=25 HN_PSNR_TAIL=1.0 HN_PSNR_LR_SCALE=$LR HN_PSNR_OUT=$OUT/short_lr${LR}_seed$S.json \
      timeout -k 10 300 python -u -m pytest tests/test_psnr.py -q -s -p no:cacheprovider --timeout 280 \
      --timeout-method thread > $OUT/short_lr${LR}_seed$S.log 2>&1
    RC=$?
    echo "lr $LR seed $S rc=$RC: $(grep '^{' $OUT/short_lr${LR}_seed$S.log | tail -1 | cut -c1-160)"
    [ $RC -le 1 ] || exit $RC
  done
done
