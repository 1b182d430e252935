#!/bin/bash
set -o pipefail
TAG=${1:-r06h}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1; RC=$?
tail -3 $O/pytest_gpu.log; [ $RC -eq 0 ] || exit $RC
PROF=1 scripts/gpu_ab3.sh $TAG "skip1:skip1.so:" "bal:-:" "baldense:-:--dense-bwd"
