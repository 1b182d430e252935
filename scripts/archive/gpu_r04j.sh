set -o pipefail
mkdir -p gpurun_out/r04j
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04j/pytest_gpu.log 2>&1; RC=$?
tail -2 gpurun_out/r04j/pytest_gpu.log; [ $RC -eq 0 ] || exit $RC
HN_LIB_PATH=hashnerf-pytorch_amd/build/var_prof_cmp.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/r04j/prof.json 2> gpurun_out/r04j/prof.err || exit 1
grep hn_fwd_profile gpurun_out/r04j/prof.err | tail -2
REPS=2 PROF=1 bash scripts/gpu_lib_ab.sh r04j var_tw var_cmp var_cmpxp || exit 1
timeout -k 10 300 python scripts/bin_stats.py --quick --dups > gpurun_out/r04j/bin_dups_config2.txt 2>&1 || { tail -5 gpurun_out/r04j/bin_dups_config2.txt; exit 1; }
cat gpurun_out/r04j/bin_dups_config2.txt
