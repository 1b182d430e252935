#!/bin/bash
# GPU job: configs 3 and 5 bench lines, a 2-rank gloo rehearsal of the DP
# path on the one GPU, and the 5k-iteration PSNR parity run.
#   usage: scripts/gpu_configs.sh TAG
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python bench.py --config 3 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_config3_$TAG.json 2> $OUT/bench_config3_$TAG.err && \
timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_config5_$TAG.json 2> $OUT/bench_config5_$TAG.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 5 --warmup 2 --pretrain 20 --backend gloo > $OUT/bench_gloo2_$TAG.json 2> $OUT/bench_gloo2_$TAG.err && \
HN_PSNR_ITERS=5000 HN_PSNR_EVERY=100 HN_PSNR_RES=200 HN_PSNR_NTRAIN=100 HN_PSNR_SEEDS=3 HN_PSNR_OUT=$OUT/psnr_5k_$TAG.json \
    timeout -k 10 1000 python -u -m pytest tests/test_psnr.py -v -s --timeout 980 --timeout-method thread > $OUT/psnr_5k_$TAG.log 2>&1
RC=$?
tail -3 $OUT/psnr_5k_$TAG.log
for f in $OUT/bench_config3_$TAG.json $OUT/bench_config5_$TAG.json $OUT/bench_gloo2_$TAG.json; do
  python -c "import json;d=json.load(open('$f'));print('$f', d['value'], d['ms_per_step'], d.get('kernels'))" || true
done
exit $RC
