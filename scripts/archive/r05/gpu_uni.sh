#!/bin/bash
set -o pipefail
O=gpurun_out/uni; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rf --timeout 170 --timeout-method thread -k "uniform_philox or sample_batch" > $O/pytest1.log 2>&1; RC=$?
tail -3 $O/pytest1.log; [ $RC -eq 0 ] || exit $RC
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 170 --timeout-method thread > $O/pytest.log 2>&1; RC=$?
tail -3 $O/pytest.log; [ $RC -eq 0 ] || exit $RC
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 > $O/b_$r.json 2>$O/err || { tail -5 $O/err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/b_$r.json
done
