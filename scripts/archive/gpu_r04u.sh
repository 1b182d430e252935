set -o pipefail
# 8-rank gloo rehearsal of the bench's data-parallel path on one GPU (world 8:
# the segmented exchange's bin/rank arithmetic at the driver's largest N), then
# 4 ranks at config 5
mkdir -p gpurun_out/r04u
timeout -k 10 600 python bench.py --gpus 8 --backend gloo --steps 2 --warmup 1 --pretrain 20 --no-cpu-baseline > gpurun_out/r04u/bench_gloo8.json 2> gpurun_out/r04u/bench_gloo8.err || { tail -8 gpurun_out/r04u/bench_gloo8.err; exit 1; }
cut -c1-220 gpurun_out/r04u/bench_gloo8.json
timeout -k 10 600 python bench.py --gpus 4 --backend gloo --config 5 --steps 3 --warmup 1 --pretrain 20 --no-cpu-baseline > gpurun_out/r04u/bench_gloo4_config5.json 2> gpurun_out/r04u/bench_gloo4_config5.err || { tail -8 gpurun_out/r04u/bench_gloo4_config5.err; exit 1; }
cut -c1-220 gpurun_out/r04u/bench_gloo4_config5.json
