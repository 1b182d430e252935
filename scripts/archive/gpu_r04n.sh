set -o pipefail
# batched-probe merge table (build/var_mb.so): scatter tests on it, then the
# merged-level breakdown against the unmerged scatter, config 2 and config 3
mkdir -p gpurun_out/r04n
export TMPDIR=/tmp
V=hashnerf-pytorch_amd/build/var_mb.so
HN_LIB_PATH=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_scatter.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04n/pytest_scatter.log 2>&1; RC=$?
tail -2 gpurun_out/r04n/pytest_scatter.log; [ $RC -eq 0 ] || exit $RC
for C in m0:0: m4:4: m7:7: m10:10: c3m0:0:--config=3 c3m8:8:--config=3; do
  N=${C%%:*}; R=${C#*:}; M=${R%%:*}; A=${R#*:}
  HN_LIB_PATH=$V HN_SC_MERGE_LEVELS=$M timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04n/prof_$N -o prof -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline $A > gpurun_out/r04n/prof_$N.log 2>&1 || { tail -5 gpurun_out/r04n/prof_$N.log; exit 1; }
  F=$(find gpurun_out/r04n/prof_$N -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_tail_stats.py $F 10 > gpurun_out/r04n/kernel_stats_$N.csv && rm -rf gpurun_out/r04n/prof_$N
  grep -h "scatter_bins\|bin_reduce" gpurun_out/r04n/kernel_stats_$N.csv | cut -d, -f1,2,4 | sed "s/^/$N /"
done
