#!/bin/bash
# Paired PSNR@5k runs (HIP trainer vs the reference path, tests/test_psnr.py)
# at several seeds IN PARALLEL on the one GPU (the reference path is bound by
# its eager launches on the host, one core each), then the aggregate with its
# 95 % CI (scripts/psnr_aggregate.py).
#   usage: scripts/gpu_psnr_multi.sh TAG SEED0 SEED1 ...
set -o pipefail
TAG=$1
shift
OUT=gpurun_out/psnr_$TAG
mkdir -p $OUT
# at most PAR runs at once (6 in parallel take ~260 s each on one box; 12
# at once were >4x slower per run: r03f reached iteration 2000 of 5000 in 18 min)
PAR=${HN_PSNR_PAR:-6}
RC=0
run_batch() {
  local PIDS=()
  for S in "$@"; do
    HN_PSNR_SEED=$S HN_PSNR_TAIL=${HN_PSNR_TAIL:-0.2} HN_PSNR_ITERS=5000 HN_PSNR_EVERY=${HN_PSNR_EVERY:-100} HN_PSNR_RES=200 HN_PSNR_NTRAIN=100 HN_PSNR_NTEST=8 \
    HN_PSNR_OUT=$OUT/psnr_5k_${TAG}_seed$S.json OMP_NUM_THREADS=1 \
        timeout -k 10 ${HN_PSNR_TIMEOUT:-540} python -u -m pytest tests/test_psnr.py -q -s -p no:cacheprovider \
        > $OUT/psnr_5k_${TAG}_seed$S.log 2>&1 &
    PIDS+=($!)
  done
  # heartbeat: the runs print every 500 iterations only (gpurun takes 180 s
  # without output for a hang)
  ( while true; do sleep 60; echo "[$(date +%T)] $(tail -qn1 $OUT/psnr_5k_${TAG}_seed$1.log 2>/dev/null | cut -c1-80)"; done ) &
  local HB=$!
  for P in "${PIDS[@]}"; do wait $P || RC=$?; done
  kill $HB 2>/dev/null
}
SEEDS=("$@")
for ((i = 0; i < ${#SEEDS[@]}; i += PAR)); do
  run_batch "${SEEDS[@]:i:PAR}"
  echo "batch $i rc=$RC"
  # a run past its limit (124/137) or killed: start nothing more
  [ $RC -eq 124 ] || [ $RC -eq 137 ] || [ $RC -gt 128 ] && break
done
echo "runs rc=$RC"
ls $OUT/*.json > /dev/null 2>&1 && python scripts/psnr_aggregate.py $OUT/psnr_5k_${TAG}.json $OUT/psnr_5k_${TAG}_seed*.json
exit $RC
