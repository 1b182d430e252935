#!/bin/bash
# r03v: validation of the round-3 final library (HN_FWD_C0SH, live-pair mask,
# dW slab reduction inside the scatter kernel): GPU tests, smoke, forward
# determinism, PMC passes -> the bench line's traffic json, the default bench
# (CPU baseline included), kernel stats over the timed steps, configs 3 and 5,
# the 2-rank gloo launcher rehearsal.
set -o pipefail
TAG=${1:-r03v}
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu_$TAG.log 2>&1
RC=$?; echo "pytest rc=$RC"; grep -E "passed|failed" $OUT/pytest_gpu_$TAG.log | tail -3; grep FAILED $OUT/pytest_gpu_$TAG.log | head
[ $RC -le 1 ] || exit $RC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || exit 2
timeout -k 10 300 python -u scripts/diag_fwd_det.py 4096 16 > $OUT/diag_fwd_det_$TAG.log 2>&1 || exit 2
echo "fwd repeats identical: $(grep -c identical $OUT/diag_fwd_det_$TAG.log) of 15"
timeout -k 10 600 bash scripts/gpu_pmc.sh $TAG > $OUT/pmc_$TAG.out 2>&1 || exit 7
cp $OUT/traffic_$TAG.json profiles/traffic_config2_procedural_p1000_binned.json
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit 3
cat $OUT/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o prof -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 || exit 5
python3 scripts/trace_tail_stats.py $OUT/prof_$TAG/prof_kernel_trace.csv 10 > $OUT/prof_$TAG/prof_kernel_stats_timed.csv
rm -f $OUT/prof_$TAG/prof_kernel_trace.csv
head -14 $OUT/prof_$TAG/prof_kernel_stats_timed.csv | cut -c1-110
for C in 3 5; do
  timeout -k 10 600 python bench.py --config $C --no-cpu-baseline > $OUT/bench_config${C}_$TAG.json 2> $OUT/bench_config${C}_$TAG.err || exit 4
  python -c "import json;d=json.load(open('$OUT/bench_config${C}_$TAG.json'));print('config$C', d['value'], d['ms_per_step'], d['kernels'])"
done
timeout -k 10 600 python bench.py --gpus 2 --backend gloo --steps 10 --pretrain 100 --no-cpu-baseline \
    > $OUT/bench_gloo2_$TAG.json 2> $OUT/bench_gloo2_$TAG.err || exit 6
python -c "import json;d=json.load(open('$OUT/bench_gloo2_$TAG.json'));print('gloo2', d['n_gpus'], d['value'], d['ms_per_step'])"
echo "chain ok"
# A/B (one box): the forward's ReLU mask bits through an inline v_min_u32
# (HN_MASK_ASM=1: 2 VALU per register instead of 3; identical bits)
for R in 1 2; do
  for V in base var_maskasm var_brrev; do
    if [ $V = base ]; then unset HN_LIB_PATH; else export HN_LIB_PATH=hashnerf-pytorch_amd/build/$V.so; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/ab_${V}_${TAG}_$R.json 2> $OUT/ab_${V}_${TAG}_$R.err || exit 8
    python -c "import json;d=json.load(open('$OUT/ab_${V}_${TAG}_$R.json'));print('$V', d['value'], d['ms_per_step'], d['kernels']['render_fwd_ms'], d['kernels']['render_bwd_ms'])"
  done
done
unset HN_LIB_PATH
echo "ab ok"
