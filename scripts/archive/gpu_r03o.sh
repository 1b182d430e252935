#!/bin/bash
# r03o: validation of the round-3 defaults (stored ReLU masks + 2-part
# recompute, one tile copy, rolled scatter levels, staged records).  GPU
# tests, smoke, PMC passes -> the bench line's traffic json, the default
# bench (CPU baseline included), kernel stats, config 3, 2-rank gloo launcher.
set -o pipefail
TAG=r03o
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu_$TAG.log 2>&1
RC=$?; echo "pytest rc=$RC"; grep -E "passed|failed" $OUT/pytest_gpu_$TAG.log | tail -3
[ $RC -le 1 ] || exit $RC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || exit 2
timeout -k 10 600 bash scripts/gpu_pmc.sh $TAG > $OUT/pmc_$TAG.out 2>&1 || exit 7
cp $OUT/traffic_$TAG.json profiles/traffic_config2_procedural_p1000_binned.json
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit 3
cat $OUT/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o prof -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 || exit 5
python3 scripts/trace_tail_stats.py $OUT/prof_$TAG/prof_kernel_trace.csv 10 > $OUT/prof_$TAG/prof_kernel_stats_timed.csv
rm -f $OUT/prof_$TAG/prof_kernel_trace.csv
head -12 $OUT/prof_$TAG/prof_kernel_stats_timed.csv | cut -c1-110
timeout -k 10 600 python bench.py --config 3 --no-cpu-baseline > $OUT/bench_config3_$TAG.json 2> $OUT/bench_config3_$TAG.err || exit 4
python -c "import json;d=json.load(open('$OUT/bench_config3_$TAG.json'));print('config3', d['value'], d['ms_per_step'], d['kernels'])"
timeout -k 10 600 python bench.py --gpus 2 --backend gloo --steps 10 --pretrain 100 --no-cpu-baseline \
    > $OUT/bench_gloo2_$TAG.json 2> $OUT/bench_gloo2_$TAG.err || exit 6
python -c "import json;d=json.load(open('$OUT/bench_gloo2_$TAG.json'));print('gloo2', d['n_gpus'], d['value'], d['ms_per_step'])"
echo "chain ok"
