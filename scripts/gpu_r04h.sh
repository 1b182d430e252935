set -o pipefail
mkdir -p gpurun_out/r04h
timeout -k 10 300 scripts/hazard/scratch_probe 40 > gpurun_out/r04h/scratch_probe.txt 2>&1 || { echo "scratch probe failed"; cat gpurun_out/r04h/scratch_probe.txt; exit 1; }
tail -3 gpurun_out/r04h/scratch_probe.txt
timeout -k 10 900 bash scripts/gpu_fwd_pmc.sh r04h_fwdpmc > gpurun_out/r04h/fwd_pmc.txt 2>&1; echo "fwd pmc rc=$?"; tail -40 gpurun_out/r04h/fwd_pmc.txt
SEEDS="0 1 2 3 4 5" LRS="1 0.7" timeout -k 10 1000 bash scripts/gpu_psnr_short_cal.sh r04h
