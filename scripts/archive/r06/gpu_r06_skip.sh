#!/bin/bash
# Round 6: exact-zero skipping -- the skip test + GPU tests, then interleaved
# bench lines with and without it (--dense-bwd) and rocprof kernel stats.
set -o pipefail
TAG=${1:-r06e}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_driver.py -x -q -rf -k zero_gradient --timeout 250 --timeout-method thread > $O/pytest_skip.log 2>&1; RC=$?
tail -3 $O/pytest_skip.log; [ $RC -eq 0 ] || exit $RC
for r in 1 2; do
  for V in dense skip; do
    A=""; [ $V = dense ] && A="--dense-bwd"
    timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline $A $BENCH_ARGS > $O/b_${V}_$r.json 2> $O/b_${V}_$r.err || { tail -5 $O/b_${V}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b_${V}_$r.json'));print('$V', $r, d['value'], d['ms_per_step'], d['kernels']['render_fwd_ms'], d['kernels']['render_bwd_ms'])"
  done
done
for V in dense skip; do
  A=""; [ $V = dense ] && A="--dense-bwd"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$V -o prof -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline $A $BENCH_ARGS > $O/prof_$V.log 2>&1 || { tail -5 $O/prof_$V.log; exit 1; }
  F=$(find $O/prof_$V -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_tail_stats.py $F 10 > $O/kernel_stats_$V.csv && rm -rf $O/prof_$V
  head -6 $O/kernel_stats_$V.csv | cut -d, -f1-4 | sed "s/^/$V /"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1; RC=$?
tail -3 $O/pytest_gpu.log; exit $RC
