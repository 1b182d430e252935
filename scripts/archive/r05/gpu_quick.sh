#!/bin/bash
# Quick GPU iteration: rebuild, GPU parity tests, short bench (no CPU baseline).
set -o pipefail
TAG=${1:-q}
OUT=gpurun_out
mkdir -p $OUT
python hashnerf-pytorch_amd/build.py > $OUT/build_$TAG.log 2>&1 || { echo "build failed"; tail $OUT/build_$TAG.log; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -x > $OUT/pytest_gpu_$TAG.log 2>&1
RC=$?
echo "pytest rc=$RC"
tail -5 $OUT/pytest_gpu_$TAG.log
# 0 = pass, 1 = test failures: the GPU is fine, go on; anything else (abort,
# segfault, timeout) ends the call
[ $RC -le 1 ] || exit $RC
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
echo "bench rc=$?"
python -c "import json;d=json.load(open('$OUT/bench_$TAG.json'));print(d['value'], d['ms_per_step'], d['kernels'])"
