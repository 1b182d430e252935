#!/bin/bash
# round-3 final check of the committed tree: GPU tests, smoke, the default
# bench line (traffic from the committed pmc_r03v json).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu_r03final.log 2>&1
RC=$?; echo "pytest rc=$RC"; tail -2 $OUT/pytest_gpu_r03final.log
[ $RC -le 1 ] || exit $RC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r03final.log 2>&1 || exit 2
tail -1 $OUT/smoke_r03final.log
timeout -k 10 600 python bench.py > $OUT/bench_r03final.json 2> $OUT/bench_r03final.err || exit 3
cat $OUT/bench_r03final.json
