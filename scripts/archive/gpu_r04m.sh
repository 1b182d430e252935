set -o pipefail
# merge table with 4,096 slots and read-before-CAS inserts: scatter tests,
# then the per-level-count breakdown
mkdir -p gpurun_out/r04m
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_scatter.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04m/pytest_scatter.log 2>&1; RC=$?
tail -2 gpurun_out/r04m/pytest_scatter.log; [ $RC -eq 0 ] || exit $RC
L=hashnerf-pytorch_amd/lib/libhashnerf_amd.so
for C in m0:$L:0 m7:$L:7 m10:$L:10; do
  N=${C%%:*}; R=${C#*:}; LIB=${R%%:*}; M=${R##*:}
  HN_LIB_PATH=$LIB HN_SC_MERGE_LEVELS=$M timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04m/prof_$N -o prof -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04m/prof_$N.log 2>&1 || { tail -5 gpurun_out/r04m/prof_$N.log; exit 1; }
  F=$(find gpurun_out/r04m/prof_$N -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_tail_stats.py $F 10 > gpurun_out/r04m/kernel_stats_$N.csv && rm -rf gpurun_out/r04m/prof_$N
  grep -h "scatter_bins\|bin_reduce" gpurun_out/r04m/kernel_stats_$N.csv | cut -d, -f1,2,4 | sed "s/^/$N /"
  grep -h '"ms_per_step"' gpurun_out/r04m/prof_$N.log | head -1 | cut -c1-20 || true
done
