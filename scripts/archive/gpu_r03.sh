#!/bin/bash
# Round-3 GPU job: GPU tests, smoke, N=1 bench, 2-rank gloo rehearsal of the
# bench launcher, rocprofv3 kernel stats of the timed steps.  Each GPU step has
# its own time limit; the chain stops at the first abort / fault / timeout.
#   usage: scripts/gpu_r03.sh TAG [pytest selection...]
set -o pipefail
TAG=${1:-r03}
shift
SEL=${*:-tests}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $SEL -m gpu -v -rf --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu_$TAG.log 2>&1
RC=$?
echo "pytest rc=$RC" | tee -a $OUT/pytest_gpu_$TAG.log
grep -E "passed|failed|error" $OUT/pytest_gpu_$TAG.log | tail -3
[ $RC -le 1 ] || exit $RC     # abort / segfault / timeout: nothing more on the GPU
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || exit 2
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit 3
cat $OUT/bench_$TAG.json
timeout -k 10 600 python bench.py --gpus 2 --backend gloo --steps 10 --pretrain 100 --no-cpu-baseline \
    > $OUT/bench_gloo2_$TAG.json 2> $OUT/bench_gloo2_$TAG.err || exit 4
cat $OUT/bench_gloo2_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o prof -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 || exit 5
python3 scripts/trace_tail_stats.py $OUT/prof_$TAG/prof_kernel_trace.csv 10 > $OUT/prof_$TAG/prof_kernel_stats_timed.csv
rm -f $OUT/prof_$TAG/prof_kernel_trace.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/prof_$TAG/prof_kernel_stats_timed.csv')))[:16]:
    print(f'{float(r[\"AverageNs\"])/1e3:9.2f} us  {r[\"Name\"][:90]}')"
echo "chain ok"
