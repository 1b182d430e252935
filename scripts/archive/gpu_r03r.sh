#!/bin/bash
# r03r: the render forward's rare nondeterminism, second bisect: the debug
# build dumps coarse tile 0's sh8 / s1 registers (in place of the mask words)
# so the glitch's first wrong value shows; the tail-nop build pads every
# GEMM's last MFMA with 16 wait states (an MFMA-read hazard would vanish).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for V in var_dbg var_tailnop; do
  export HN_LIB_PATH=hashnerf-pytorch_amd/build/$V.so
  timeout -k 10 300 python -u scripts/diag_fwd_det.py 4096 16 > $OUT/diag_fwd_det_${V}_r03r.log 2>&1 || exit 2
  echo "== $V"; grep -v amdgpu.ids $OUT/diag_fwd_det_${V}_r03r.log | cut -c1-900
done
echo "chain ok"
