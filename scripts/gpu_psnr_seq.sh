#!/bin/bash
# Paired PSNR@5k runs one after another (tests/test_psnr.py; parallel runs on
# one GPU slowed each run ~5x in r03x).  Seeds named "cN" re-run only the HIP
# side against the cached reference curve of run N's earlier paired JSON
# (HN_PSNR_REF_CACHE; profiles/r03/psnr_r03y/psnr_5k_r03y_seedN.json, or
# PSNR_CACHE_GLOB).
#   usage: scripts/gpu_psnr_seq.sh TAG SEED|cSEED ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/psnr_$TAG; mkdir -p $OUT
for S in "$@"; do
  C=""
  if [ "${S:0:1}" = c ]; then S=${S:1}; C=$(ls ${PSNR_CACHE_GLOB:-profiles/r03/psnr_r03y/psnr_5k_r03y_seed}$S.json | head -1); fi
  HN_PSNR_SEED=$S HN_PSNR_TAIL=0.2 HN_PSNR_ITERS=5000 HN_PSNR_EVERY=100 HN_PSNR_RES=200 HN_PSNR_NTRAIN=100 \
  HN_PSNR_NTEST=8 HN_PSNR_OUT=$OUT/psnr_5k_${TAG}_seed$S.json HN_PSNR_REF_CACHE=$C \
      timeout -k 10 ${HN_PSNR_TIMEOUT:-480} python -u -m pytest tests/test_psnr.py -k test_psnr_parity_equal_iterations \
      -q -s -p no:cacheprovider \
      > $OUT/psnr_5k_${TAG}_seed$S.log 2>&1
  RC=$?
  echo "seed $S (cache: ${C:-none}) rc=$RC: $(grep '^{' $OUT/psnr_5k_${TAG}_seed$S.log | tail -1 | cut -c1-200)"
  [ $RC -le 1 ] || exit $RC
done
