set -o pipefail
# calibration of the short PSNR gate (tests/test_psnr.py): paired 400-iteration runs, and the same with the HIP side's lr x 0.7
SEEDS="0 1 2 3 4 5" LRS="1 0.7" timeout -k 10 1100 bash scripts/gpu_psnr_short_cal.sh r04i
