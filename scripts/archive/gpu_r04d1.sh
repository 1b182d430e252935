#!/bin/bash
# MFMA hazard probes; configs 3 and 5 made measurable like config 2: PMC
# traffic + MFMA busy and rocprofv3 kernel stats.
set -o pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT
export TMPDIR=/tmp
# MFMA operand-hazard probes (scripts/hazard/*.hip, built on the CPU side)
timeout -k 10 180 scripts/hazard/mfma_hazard 20 > $OUT/mfma_hazard.txt 2>&1 || { echo "hazard probe failed"; cat $OUT/mfma_hazard.txt; exit 1; }
cat $OUT/mfma_hazard.txt
timeout -k 10 180 scripts/hazard/mfma_overlap 20 > $OUT/mfma_overlap.txt 2>&1 || { echo "overlap probe failed"; exit 1; }
tail -1 $OUT/mfma_overlap.txt
for C in 3 5; do
  timeout -k 10 900 bash scripts/gpu_pmc.sh c${C}_r04d --config $C > $OUT/pmc_c$C.txt 2>&1 || { echo "pmc config $C failed"; tail -3 $OUT/pmc_c$C.txt; exit 1; }
  cp gpurun_out/traffic_c${C}_r04d.json profiles/traffic_config${C}_procedural_p1000_binned.json
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_c$C -o prof -- \
      python3 bench.py --config $C --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_c$C.log 2>&1 || { echo "trace $C failed"; exit 1; }
  python3 scripts/trace_tail_stats.py $(find $OUT/prof_c$C -name "*kernel_trace.csv" | head -1) 10 > $OUT/kernel_stats_config${C}_r04d.csv && rm -rf $OUT/prof_c$C
  head -8 $OUT/kernel_stats_config${C}_r04d.csv | cut -d, -f1-4
done
