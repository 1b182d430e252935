#!/bin/bash
set -o pipefail
TAG=${1:-r06ab}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 scripts/hazard/div_rn_check > $O/div_rn_check.txt 2>&1; RC=$?; cat $O/div_rn_check.txt; [ $RC -eq 0 ] || exit $RC
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1; RC=$?
tail -2 $O/pytest_gpu.log; [ $RC -eq 0 ] || exit $RC
PROF=1 scripts/gpu_ab3.sh $TAG "pairs:pairs.so:" "divrn:-:"
