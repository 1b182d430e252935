#!/bin/bash
# r03t: HN_FWD_C0SH (color_net.0's SH half once per ray from LDS) as the
# default: forward determinism over 32 repeats, the GPU tests, then the
# live-pair mask A/B (config 2 x2, config 3) with the host-enqueue figure.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/diag_fwd_det.py 4096 32 > $OUT/diag_fwd_det_r03t.log 2>&1 || exit 2
echo "fwd repeats identical: $(grep -c identical $OUT/diag_fwd_det_r03t.log) of 31"; grep -v "amdgpu.ids\|identical" $OUT/diag_fwd_det_r03t.log | cut -c1-300
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu_r03t.log 2>&1
RC=$?; echo "pytest rc=$RC"; grep -E "passed|failed" $OUT/pytest_gpu_r03t.log | tail -3; grep FAILED $OUT/pytest_gpu_r03t.log | head
[ $RC -le 1 ] || exit $RC
for R in 1 2; do
  for V in mask dense; do
    F=""; [ $V = dense ] && F="--dense-table-step"
    timeout -k 10 300 python bench.py --no-cpu-baseline $F > $OUT/ab_${V}_$R.json 2> $OUT/ab_${V}_$R.err || exit 4
    python -c "import json;d=json.load(open('$OUT/ab_${V}_$R.json'));print('c2 $V', d['value'], d['ms_per_step'], d['kernels'], 'host', d['host_enqueue_ms'])"
  done
done
for V in mask dense; do
  F=""; [ $V = dense ] && F="--dense-table-step"
  timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline $F > $OUT/ab3_${V}.json 2> $OUT/ab3_${V}.err || exit 5
  python -c "import json;d=json.load(open('$OUT/ab3_${V}.json'));print('c3 $V', d['value'], d['ms_per_step'], d['kernels'], 'host', d['host_enqueue_ms'])"
done
echo "chain ok"
