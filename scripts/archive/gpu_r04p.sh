set -o pipefail
# PMC traffic / MFMA busy of config 2 at HEAD (all default passes), and a
# 2-rank gloo rehearsal of the bench's data-parallel path (segmented exchange)
mkdir -p gpurun_out/r04p
export TMPDIR=/tmp
timeout -k 10 900 bash scripts/gpu_pmc.sh r04p > gpurun_out/r04p/pmc.txt 2>&1; echo "pmc rc=$?"
grep -A6 "render_fwd_kernel\|scatter_bins\|bin_reduce" gpurun_out/r04p/pmc.txt | head -40
timeout -k 10 600 python bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04p/bench_gloo2.json 2> gpurun_out/r04p/bench_gloo2.err; echo "gloo2 rc=$?"
cut -c1-200 gpurun_out/r04p/bench_gloo2.json
