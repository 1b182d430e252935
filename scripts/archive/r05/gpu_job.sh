#!/bin/bash
# GPU job used with gpurun: tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; the chain stops at the first failure.
#   usage: scripts/gpu_job.sh [tag] [steps]
set -o pipefail
TAG=${1:-r01}
STEPS=${2:-20}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
python hashnerf-pytorch_amd/build.py > $OUT/build_$TAG.log 2>&1 || { echo "build failed"; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > $OUT/pytest_gpu_$TAG.log 2>&1
RC=$?
echo "pytest rc=$RC" | tee -a $OUT/pytest_gpu_$TAG.log
tail -4 $OUT/pytest_gpu_$TAG.log
[ $RC -le 1 ] || exit $RC     # abort / segfault / timeout: nothing more on the GPU
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 && \
timeout -k 10 600 python bench.py --steps $STEPS --warmup 5 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err && \
cat $OUT/bench_$TAG.json && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o prof -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1
RC=$?
# the timed steps only (the 13 last dispatches of each kernel: 3 warmup + 10 timed)
[ $RC -eq 0 ] && python3 scripts/trace_tail_stats.py $OUT/prof_$TAG/prof_kernel_trace.csv 10 \
    > $OUT/prof_$TAG/prof_kernel_stats_timed.csv
rm -f $OUT/prof_$TAG/prof_kernel_trace.csv   # per-dispatch rows of the pretraining too: large
echo "chain rc=$RC"
tail -3 $OUT/smoke_$TAG.log
