#!/bin/bash
# Diagnostic: per-iteration cost of paired PSNR runs (300 iterations at the
# 5k run's shape) with K of them at once on the one GPU.
set -o pipefail
OUT=gpurun_out/psnr_diag; mkdir -p $OUT
for K in ${@:-3 6}; do
  PIDS=()
  for S in $(seq 1 $K); do
    HN_PSNR_SEED=$S HN_PSNR_ITERS=300 HN_PSNR_EVERY=100 HN_PSNR_RES=200 HN_PSNR_NTRAIN=100 HN_PSNR_NTEST=8 \
    HN_PSNR_OUT=$OUT/par${K}_$S.json timeout -k 10 170 python -u -m pytest tests/test_psnr.py -q -s -p no:cacheprovider \
        > $OUT/par${K}_$S.log 2>&1 &
    PIDS+=($!)
  done
  RC=0; for P in "${PIDS[@]}"; do wait $P || RC=$?; done
  echo "K=$K rc=$RC"
  for S in $(seq 1 $K); do python -c "import json;d=json.load(open('$OUT/par${K}_$S.json'));print(d['ms_per_iter_hip'], d['ms_per_iter_ref_eager_gpu'])" 2>/dev/null || echo "seed $S: no json"; done
  [ $RC -eq 0 ] || break
done
