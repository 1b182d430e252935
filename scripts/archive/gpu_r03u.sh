#!/bin/bash
# r03u: PSNR@5k on the final round-3 library, 12 paired seeds (0-11) in two
# batches of six, tail evaluations every 50 iterations (20 in the last 20 %),
# aggregate with the 95 % CI (scripts/psnr_aggregate.py).
set -o pipefail
export TMPDIR=/tmp
HN_PSNR_EVERY=50 HN_PSNR_TIMEOUT=760 bash scripts/gpu_psnr_multi.sh r03u 0 1 2 3 4 5 6 7 8 9 10 11
