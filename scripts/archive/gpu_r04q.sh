set -o pipefail
# PSNR@5k of the round-4 library: the HIP side of 12 paired seeds re-run
# against the reference curves of round 3's runs (the reference path is a
# function of the seed alone; copies of those curves in profiles/r04/psnr_ref_r03y)
PSNR_CACHE_GLOB=profiles/r04/psnr_ref_r03y/psnr_5k_r03y_seed HN_PSNR_TIMEOUT=150 timeout -k 10 1100 bash scripts/gpu_psnr_seq.sh r04q c0 c1 c2 c3 c4 c5 c6 c7 c8 c9 c10 c11
