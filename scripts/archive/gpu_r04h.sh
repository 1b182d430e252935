set -o pipefail
mkdir -p gpurun_out/r04h
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04h/pytest_gpu.log 2>&1; RC=$?
tail -2 gpurun_out/r04h/pytest_gpu.log; [ $RC -eq 0 ] || exit $RC
REPS=2 PROF=1 bash scripts/gpu_lib_ab.sh r04h var_base2 var_tw var_xp2 || exit 1
timeout -k 10 300 scripts/hazard/scratch_probe 40 > gpurun_out/r04h/scratch_probe.txt 2>&1 || { echo "scratch probe failed"; cat gpurun_out/r04h/scratch_probe.txt; exit 1; }
tail -3 gpurun_out/r04h/scratch_probe.txt
timeout -k 10 900 bash scripts/gpu_fwd_pmc.sh r04h_fwdpmc > gpurun_out/r04h/fwd_pmc.txt 2>&1; echo "fwd pmc rc=$?"; tail -40 gpurun_out/r04h/fwd_pmc.txt
