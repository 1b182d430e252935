set -o pipefail
mkdir -p gpurun_out/r04b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04b/pytest_gpu.log 2>&1; RC=$?
tail -2 gpurun_out/r04b/pytest_gpu.log; [ $RC -eq 0 ] || exit $RC
REPS=2 PROF=1 bash scripts/gpu_lib_ab.sh r04b var_enc0 var_enc1 var_enc2
