set -o pipefail
# cross-row run folding in the scatter (build/var_xrow.so): scatter + trainer
# tests on it, record counts, A/B kernel stats against the default library
mkdir -p gpurun_out/r04t
export TMPDIR=/tmp
V=hashnerf-pytorch_amd/build/var_xrow.so
HN_LIB_PATH=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_scatter.py tests/test_gpu_driver.py -x -q -rf --timeout 150 --timeout-method thread > gpurun_out/r04t/pytest.log 2>&1; RC=$?
tail -2 gpurun_out/r04t/pytest.log; [ $RC -eq 0 ] || exit $RC
HN_LIB_PATH=$V timeout -k 10 300 python scripts/bin_stats.py --quick > gpurun_out/r04t/bin_counts_xrow.txt 2>&1 || { tail -3 gpurun_out/r04t/bin_counts_xrow.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04t/bin_counts_xrow.txt | head -3
for r in 1 2; do
for C in base:hashnerf-pytorch_amd/lib/libhashnerf_amd.so xrow:$V; do
  N=${C%%:*}; LIB=${C#*:}
  HN_LIB_PATH=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04t/prof_$N -o prof -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04t/prof_${N}_$r.log 2>&1 || { tail -5 gpurun_out/r04t/prof_${N}_$r.log; exit 1; }
  F=$(find gpurun_out/r04t/prof_$N -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_tail_stats.py $F 10 > gpurun_out/r04t/kernel_stats_${N}_$r.csv && rm -rf gpurun_out/r04t/prof_$N
  grep -h "scatter_bins\|bin_reduce" gpurun_out/r04t/kernel_stats_${N}_$r.csv | cut -d, -f1,2,4 | sed "s/^/$N $r /"
done
done
