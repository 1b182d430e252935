set -o pipefail
# configs 3, 5 and 4 on the final library (bench lines with the CPU baseline at each config's B)
mkdir -p gpurun_out/r04cfg
for C in 3 5 4; do
  timeout -k 10 300 python bench.py --config $C > gpurun_out/r04cfg/bench_config${C}_final.json 2> gpurun_out/r04cfg/bench_config${C}_final.err || { echo "bench $C failed"; tail -3 gpurun_out/r04cfg/bench_config${C}_final.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04cfg/bench_config${C}_final.json'));print($C, d['value'], d['ms_per_step'], d['kernels'], d.get('cpu_baseline',{}).get('value'))"
done
