#!/bin/bash
# r03s: the render forward's rare nondeterminism, third bisect: default
# (24 identical forwards), all waitcnts forced to zero (memory-ordering races
# vanish), s_nop padding before every instruction (issue hazards vanish).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for V in default var_wz var_snop; do
  if [ $V = default ]; then unset HN_LIB_PATH; else export HN_LIB_PATH=hashnerf-pytorch_amd/build/$V.so; fi
  timeout -k 10 300 python -u scripts/diag_fwd_det.py 4096 24 > $OUT/diag_fwd_det_${V}_r03s.log 2>&1 || exit 2
  echo "== $V: $(grep -c identical $OUT/diag_fwd_det_${V}_r03s.log) identical of 23"
  grep -v "amdgpu.ids\|identical" $OUT/diag_fwd_det_${V}_r03s.log | cut -c1-300
done
echo "chain ok"
