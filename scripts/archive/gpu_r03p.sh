#!/bin/bash
# r03p: (1) is the render forward deterministic?  (the binned-vs-atomic
# MLP-gradient mismatch of r03o came from two separate forwards: diag_b_vs_a
# shows bitwise-equal coarse grads when the states match); (2) GPU tests
# (ABI 11: live-pair mask of the fused table step); (3) A/B of the mask.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/diag_fwd_det.py 4096 8 > $OUT/diag_fwd_det_r03p.log 2>&1 || exit 2
cat $OUT/diag_fwd_det_r03p.log
HN_LIB_PATH=hashnerf-pytorch_amd/build/var_nosmask.so timeout -k 10 300 python -u scripts/diag_fwd_det.py 4096 6 \
    > $OUT/diag_fwd_det_nosmask_r03p.log 2>&1 || exit 3
cat $OUT/diag_fwd_det_nosmask_r03p.log
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu_r03p.log 2>&1
RC=$?; echo "pytest rc=$RC"; grep -E "passed|failed" $OUT/pytest_gpu_r03p.log | tail -3
[ $RC -le 1 ] || exit $RC
for R in 1 2; do
  for V in mask dense; do
    F=""; [ $V = dense ] && F="--dense-table-step"
    timeout -k 10 300 python bench.py --no-cpu-baseline $F > $OUT/ab_${V}_$R.json 2> $OUT/ab_${V}_$R.err || exit 4
    python -c "import json;d=json.load(open('$OUT/ab_${V}_$R.json'));print('c2 $V', d['value'], d['ms_per_step'], d['kernels']['render_bwd_ms'])"
  done
done
for V in mask dense; do
  F=""; [ $V = dense ] && F="--dense-table-step"
  timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline $F > $OUT/ab3_${V}.json 2> $OUT/ab3_${V}.err || exit 5
  python -c "import json;d=json.load(open('$OUT/ab3_${V}.json'));print('c3 $V', d['value'], d['ms_per_step'], d['kernels']['render_bwd_ms'])"
done
echo "chain ok"
