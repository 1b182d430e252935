#!/bin/bash
# A/B: the MLP RAdam step in the backward's slab reduction vs its own launch.
set -o pipefail
O=gpurun_out/abm3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 170 --timeout-method thread -k "fused_mlp or fused_table or trainer or dp" > $O/pytest.log 2>&1; RC=$?
tail -3 $O/pytest.log; [ $RC -eq 0 ] || exit $RC
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 > $O/fused_$r.json 2>$O/err || { tail -5 $O/err; exit 1; }
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --separate-mlp-step > $O/sep_$r.json 2>$O/err || { tail -5 $O/err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/fused_$r.json $O/sep_$r.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o prof -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
F=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_tail_stats.py $F 10 > $O/kernel_stats.csv && rm -rf $O/prof
cut -d, -f1,2,4 $O/kernel_stats.csv | cut -c1-100
