#!/bin/bash
# r03k: A/B (next-unit feature prefetch; old mask bits) on the new defaults,
# then paired PSNR@5k seeds run one after the other (several processes on the
# one GPU slow each other down >5x on these boxes: gpurun_out/psnr_diag).
#   usage: scripts/gpu_r03k.sh SEED...
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for V in base var_prefetch var_maskold base var_prefetch var_maskold; do
  if [ $V = base ]; then L=hashnerf-pytorch_amd/lib/libhashnerf_amd.so; else L=hashnerf-pytorch_amd/build/$V.so; fi
  HN_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/ab_$V.json 2> $OUT/ab_$V.err || exit 6
  python -c "import json;d=json.load(open('$OUT/ab_$V.json'));print('$V', d['value'], d['ms_per_step'], d['kernels']['render_fwd_ms'], d['kernels']['render_bwd_ms'])"
done
[ $# -gt 0 ] && HN_PSNR_PAR=1 HN_PSNR_TIMEOUT=560 bash scripts/gpu_psnr_multi.sh r03k "$@"
