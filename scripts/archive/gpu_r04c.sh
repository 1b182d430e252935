set -o pipefail
mkdir -p gpurun_out/r04c
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04c/pytest_gpu.log 2>&1; RC=$?
tail -2 gpurun_out/r04c/pytest_gpu.log; [ $RC -eq 0 ] || exit $RC
HN_LIB_PATH=hashnerf-pytorch_amd/build/var_prof2.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/r04c/prof.json 2> gpurun_out/r04c/prof.err || exit 1
grep hn_fwd_profile gpurun_out/r04c/prof.err | tail -2
REPS=2 PROF=1 bash scripts/gpu_lib_ab.sh r04c var_base var_r0 var_ms var_xp var_newpair || exit 1
