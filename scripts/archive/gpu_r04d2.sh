#!/bin/bash
# Bench lines of configs 3, 5 (traffic from r04d1's PMC files) and 4 with the
# CPU baseline at the config's B, a 4-rank gloo rehearsal of configs[4], and
# the forward's L1/L2 request counters.
set -o pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $OUT/pytest_gpu_d2.log 2>&1; RC=$?
tail -2 $OUT/pytest_gpu_d2.log; [ $RC -eq 0 ] || exit $RC
for C in 3 5 4; do
  timeout -k 10 600 python bench.py --config $C > $OUT/bench_config${C}_r04d.json 2> $OUT/bench_config${C}_r04d.err || { echo "bench $C failed"; tail -3 $OUT/bench_config${C}_r04d.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_config${C}_r04d.json'));print($C, d['value'], d['ms_per_step'], d['roofline']['traffic'], d.get('cpu_baseline',{}).get('value'))"
done
timeout -k 10 600 python bench.py --gpus 4 --backend gloo --config 5 --steps 5 --warmup 2 --pretrain 20 --no-cpu-baseline \
    > $OUT/bench_gloo4_config5_r04d.json 2> $OUT/bench_gloo4_config5_r04d.err || { echo "gloo4 failed"; tail -5 $OUT/bench_gloo4_config5_r04d.err; exit 1; }
cat $OUT/bench_gloo4_config5_r04d.json | cut -c1-300
# the forward's L1/L2 request counters (config 2), last: the counter names are not verified on this pool
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
PMC_PASSES="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum;TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
    timeout -k 10 600 bash scripts/gpu_pmc.sh c2l2_r04d > $OUT/pmc_c2l2.txt 2>&1
echo "l2 pmc rc=$?"; grep -A8 "render_fwd_kernel" gpurun_out/pmc_c2l2_r04d.txt 2>/dev/null | head -8
