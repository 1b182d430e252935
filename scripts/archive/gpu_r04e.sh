set -o pipefail
mkdir -p gpurun_out/r04e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04e/pytest_gpu.log 2>&1; RC=$?
tail -2 gpurun_out/r04e/pytest_gpu.log; [ $RC -eq 0 ] || exit $RC
HN_LIB_PATH=hashnerf-pytorch_amd/build/var_ldsw_prof.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/r04e/prof.json 2> gpurun_out/r04e/prof.err || exit 1
grep hn_fwd_profile gpurun_out/r04e/prof.err | tail -2
REPS=2 PROF=1 bash scripts/gpu_lib_ab.sh r04e var_head var_l0 var_ldsw || exit 1
