set -o pipefail
# the default library with the forward's wave priority: every GPU test; then
# an A/B of the owner / scatter load priority (build/var_oprio.so)
mkdir -p gpurun_out/r04y
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 150 --timeout-method thread > gpurun_out/r04y/pytest_gpu.log 2>&1; RC=$?
tail -2 gpurun_out/r04y/pytest_gpu.log; [ $RC -eq 0 ] || exit $RC
REPS=2 PROF=1 bash scripts/gpu_lib_ab.sh r04y var_base var_oprio || exit 1
