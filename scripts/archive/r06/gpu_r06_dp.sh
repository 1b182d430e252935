#!/bin/bash
# Round 6: DP path checks on one GPU -- the DP / TV-only GPU tests, then a
# 2-rank gloo rehearsal of bench.py --gpus 2 (exchange fields).
set -o pipefail
TAG=${1:-r06b}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_scatter.py tests/test_gpu_driver.py -x -v --timeout 170 --timeout-method thread > $O/pytest.log 2>&1; RC=$?
tail -5 $O/pytest.log; [ $RC -eq 0 ] || exit $RC
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --pretrain 20 --kernel-steps 3 > $O/gloo2.json 2> $O/gloo2.err || { tail -5 $O/gloo2.err; exit 1; }
grep '^{' $O/gloo2.json | cut -c1-200
