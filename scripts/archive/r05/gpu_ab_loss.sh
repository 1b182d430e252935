#!/bin/bash
# A/B: the loss formed by the backward's pre-pass vs its own launch.
set -o pipefail
O=gpurun_out/abl; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 170 --timeout-method thread -k "fused_loss or prefetch or bitwise or deterministic" > $O/pytest.log 2>&1; RC=$?
tail -3 $O/pytest.log; [ $RC -eq 0 ] || exit $RC
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 > $O/fused_$r.json 2>$O/err || { tail -5 $O/err; exit 1; }
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --separate-loss > $O/sep_$r.json 2>$O/err || { tail -5 $O/err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/fused_$r.json $O/sep_$r.json
done
