set -o pipefail
# merged coarse-level records in the binned scatter: GPU tests, A/B against
# the same library with merging off, record counts, PMC traffic
mkdir -p gpurun_out/r04k
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04k/pytest_gpu.log 2>&1; RC=$?
tail -2 gpurun_out/r04k/pytest_gpu.log; [ $RC -eq 0 ] || exit $RC
for r in 1 2; do
  for M in auto 0; do
    if [ $M = auto ]; then unset HN_SC_MERGE_LEVELS; else export HN_SC_MERGE_LEVELS=$M; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04k/merge_${M}_$r.json 2> gpurun_out/r04k/merge_${M}_$r.err || { tail -5 gpurun_out/r04k/merge_${M}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r04k/merge_${M}_$r.json'));print('merge $M', $r, d['value'], d['ms_per_step'], d['kernels']['render_fwd_ms'], d['kernels']['render_bwd_ms'])"
  done
done
for M in auto 0; do
  if [ $M = auto ]; then unset HN_SC_MERGE_LEVELS; else export HN_SC_MERGE_LEVELS=$M; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04k/prof_$M -o prof -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04k/prof_$M.log 2>&1 || { tail -5 gpurun_out/r04k/prof_$M.log; exit 1; }
  F=$(find gpurun_out/r04k/prof_$M -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_tail_stats.py $F 10 > gpurun_out/r04k/kernel_stats_merge_$M.csv && rm -rf gpurun_out/r04k/prof_$M
  grep -h "render_fwd_kernel\|render_bwd_kernel\|scatter_bins\|bin_reduce" gpurun_out/r04k/kernel_stats_merge_$M.csv | cut -d, -f1,2,4 | sed "s/^/merge $M /"
done
unset HN_SC_MERGE_LEVELS
timeout -k 10 300 python scripts/bin_stats.py --quick > gpurun_out/r04k/bin_counts_merged.txt 2>&1 || { tail -5 gpurun_out/r04k/bin_counts_merged.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04k/bin_counts_merged.txt
PMC_PASSES="FETCH_SIZE;WRITE_SIZE" timeout -k 10 400 bash scripts/gpu_pmc.sh r04k_merged > gpurun_out/r04k/pmc.txt 2>&1; echo "pmc rc=$?"; tail -30 gpurun_out/r04k/pmc.txt
