#!/bin/bash
# r03z: PSNR@5k on the final round-3 library, paired seeds 7-10 (sequential).
set -o pipefail
export TMPDIR=/tmp
bash scripts/gpu_psnr_seq.sh r03y 7 8 9 10
