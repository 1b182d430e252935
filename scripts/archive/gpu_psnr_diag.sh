#!/bin/bash
# Diagnostic: per-iteration cost of one paired PSNR run (300 iterations at the
# 5k run's shape) with OMP_NUM_THREADS=1 and with the box default.
set -o pipefail
OUT=gpurun_out/psnr_diag; mkdir -p $OUT
for OMP in 1 default; do
  if [ $OMP = 1 ]; then export OMP_NUM_THREADS=1; else unset OMP_NUM_THREADS; fi
  HN_PSNR_SEED=0 HN_PSNR_ITERS=300 HN_PSNR_EVERY=100 HN_PSNR_RES=200 HN_PSNR_NTRAIN=100 HN_PSNR_NTEST=8 \
  HN_PSNR_OUT=$OUT/diag_omp$OMP.json timeout -k 10 400 python -u -m pytest tests/test_psnr.py -q -s -p no:cacheprovider \
      > $OUT/diag_omp$OMP.log 2>&1
  echo "omp=$OMP rc=$?"; python -c "import json;d=json.load(open('$OUT/diag_omp$OMP.json'));print(d['ms_per_iter_hip'], d['ms_per_iter_ref_eager_gpu'])"
  grep -E "passed|failed" $OUT/diag_omp$OMP.log | tail -1
done
