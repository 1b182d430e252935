#!/bin/bash
set -o pipefail
O=gpurun_out/brpf; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 170 --timeout-method thread -k "fused_table_step or bitwise or trainer" > $O/pytest.log 2>&1; RC=$?
tail -3 $O/pytest.log; [ $RC -eq 0 ] || exit $RC
REPS=2 PROF=1 scripts/gpu_lib_ab.sh brpf var_brpf0 var_brpf1 || exit 1
REPS=1 PROF=1 BENCH_ARGS="--config 3" scripts/gpu_lib_ab.sh brpf3 var_brpf0 var_brpf1
