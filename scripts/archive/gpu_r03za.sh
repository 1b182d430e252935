#!/bin/bash
# r03za: PSNR@5k on the final round-3 library, paired seeds 11-14 (sequential).
set -o pipefail
export TMPDIR=/tmp
bash scripts/gpu_psnr_seq.sh r03y ${@:-11 12 13 14}
