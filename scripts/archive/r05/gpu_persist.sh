#!/bin/bash
set -o pipefail
O=gpurun_out/persist; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_scatter.py tests/test_gpu_dp.py -m gpu -x -q -rf --timeout 170 --timeout-method thread > $O/pytest.log 2>&1; RC=$?
tail -3 $O/pytest.log; [ $RC -eq 0 ] || exit $RC
REPS=2 scripts/gpu_digest_ab.sh persist var_np var_p || exit 1
BENCH_ARGS="--config 3" REPS=1 scripts/gpu_ab_var.sh persist3 var_np var_p
