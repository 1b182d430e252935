#!/bin/bash
# r03fin: profiles of the committed round-3 tree: PMC passes -> the bench
# line's traffic json, rocprofv3 kernel stats over the timed steps, the
# default bench line.
set -o pipefail
TAG=r03fin
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 bash scripts/gpu_pmc.sh $TAG > $OUT/pmc_$TAG.out 2>&1 || exit 7
cp $OUT/traffic_$TAG.json profiles/traffic_config2_procedural_p1000_binned.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o prof -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 || exit 5
python3 scripts/trace_tail_stats.py $OUT/prof_$TAG/prof_kernel_trace.csv 10 > $OUT/prof_$TAG/prof_kernel_stats_timed.csv
rm -f $OUT/prof_$TAG/prof_kernel_trace.csv
head -14 $OUT/prof_$TAG/prof_kernel_stats_timed.csv | cut -c1-110
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit 3
python -c "import json;d=json.load(open('$OUT/bench_$TAG.json'));print('bench', d['value'], d['ms_per_step'], d['kernels'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline']['traffic_source'])"
echo "chain ok"
