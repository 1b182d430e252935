#!/bin/bash
# Diagnostic: the short PSNR parity test (400 iterations at 100x100) for a few
# seeds under each HN_SCATTER schedule; prints the final statistic per run.
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
for MODE in atomic split; do
  for SEED in ${SEEDS:-0 1 2}; do
    HN_SCATTER=$MODE HN_PSNR_SEED=$SEED timeout -k 10 200 python -u -m pytest tests/test_psnr.py -q -s \
        --timeout 180 --timeout-method thread > $OUT/psnr_${MODE}_$SEED.log 2>&1
    RC=$?
    [ $RC -le 1 ] || exit $RC
    echo "$MODE seed $SEED: $(grep -o '{"psnr_hip"[^}]*}' $OUT/psnr_${MODE}_$SEED.log)"
  done
done
