set -o pipefail
# merged-record cost breakdown (levels merged 0 / 4 / 7 / 10; table inserts
# skipped: var_mdiag) and the x-pair forward, kernel stats per case
mkdir -p gpurun_out/r04l
export TMPDIR=/tmp
L=hashnerf-pytorch_amd/lib/libhashnerf_amd.so
B=hashnerf-pytorch_amd/build
for C in m0:$L:0 m4:$L:4 m7:$L:7 m10:$L:10 diag10:$B/var_mdiag.so:10 xp0:$B/var_xp.so:0; do
  N=${C%%:*}; R=${C#*:}; LIB=${R%%:*}; M=${R##*:}
  HN_LIB_PATH=$LIB HN_SC_MERGE_LEVELS=$M timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04l/prof_$N -o prof -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04l/prof_$N.log 2>&1 || { tail -5 gpurun_out/r04l/prof_$N.log; exit 1; }
  F=$(find gpurun_out/r04l/prof_$N -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_tail_stats.py $F 10 > gpurun_out/r04l/kernel_stats_$N.csv && rm -rf gpurun_out/r04l/prof_$N
  grep -h "render_fwd_kernel\|render_bwd_kernel\|scatter_bins\|bin_reduce" gpurun_out/r04l/kernel_stats_$N.csv | cut -d, -f1,2,4 | sed "s/^/$N /"
done
