set -o pipefail
mkdir -p gpurun_out/r04g
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04g/pytest_gpu.log 2>&1; RC=$?
tail -2 gpurun_out/r04g/pytest_gpu.log; [ $RC -eq 0 ] || exit $RC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04g/smoke.log 2>&1 || exit 2
tail -1 gpurun_out/r04g/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r04g/bench.json 2> gpurun_out/r04g/bench.err || exit 3
python -c "import json;d=json.load(open('gpurun_out/r04g/bench.json'));print(d['value'], d['ms_per_step'], d['kernels'], d['cpu_baseline']['value'])"
bash scripts/gpu_r04d1.sh
