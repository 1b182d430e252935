#!/bin/bash
# Full check of the tree on one GPU: GPU tests, smoke, the default bench line.
# usage: scripts/gpu_check.sh TAG   (outputs under gpurun_out/TAG/)
set -o pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1
RC=$?; echo "pytest rc=$RC"; tail -3 $OUT/pytest_gpu.log
[ $RC -le 1 ] || exit $RC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 2
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 3
cat $OUT/bench.json
