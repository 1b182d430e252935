#!/bin/bash
# Configs 3 and 5 at HEAD: PMC traffic + MFMA busy (the files bench.py reads)
# and kernel stats; then the bench lines of configs 3, 5 and 4 with the CPU
# baseline at each config's B.
set -o pipefail
OUT=gpurun_out/r04r; mkdir -p $OUT
export TMPDIR=/tmp
for C in 3 5; do
  timeout -k 10 400 bash scripts/gpu_pmc.sh c${C}_r04r --config $C > $OUT/pmc_c$C.txt 2>&1 || { echo "pmc config $C failed"; tail -3 $OUT/pmc_c$C.txt; exit 1; }
  cp gpurun_out/traffic_c${C}_r04r.json profiles/traffic_config${C}_procedural_p1000_binned.json
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_c$C -o prof -- \
      python3 bench.py --config $C --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_c$C.log 2>&1 || { echo "trace $C failed"; exit 1; }
  python3 scripts/trace_tail_stats.py $(find $OUT/prof_c$C -name "*kernel_trace.csv" | head -1) 10 > $OUT/kernel_stats_config${C}_r04r.csv && rm -rf $OUT/prof_c$C
  head -6 $OUT/kernel_stats_config${C}_r04r.csv | cut -d, -f1-4
done
for C in 3 5 4; do
  timeout -k 10 300 python bench.py --config $C > $OUT/bench_config${C}_r04r.json 2> $OUT/bench_config${C}_r04r.err || { echo "bench $C failed"; tail -3 $OUT/bench_config${C}_r04r.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_config${C}_r04r.json'));print($C, d['value'], d['ms_per_step'], d['roofline']['traffic'], d.get('cpu_baseline',{}).get('value'))"
done
