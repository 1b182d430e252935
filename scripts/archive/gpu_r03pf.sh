#!/bin/bash
# r03pf: HN_GEMM_PF=0 (the new default) against the prefetching build
# (var_pf1): forward state and backward gradients bitwise; then the GPU tests
# and the default bench line of the committed tree.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/diag_fwd_dump.py $OUT/state_pf0.npz > $OUT/dump_pf0.log 2>&1 || exit 2
HN_LIB_PATH=hashnerf-pytorch_amd/build/var_pf1.so timeout -k 10 200 python -u scripts/diag_fwd_dump.py $OUT/state_pf1.npz > $OUT/dump_pf1.log 2>&1 || exit 2
python - <<'PY' | tee $OUT/pf_bitwise_r03pf.txt
import numpy as np
a, b = np.load("gpurun_out/state_pf0.npz"), np.load("gpurun_out/state_pf1.npz")
for k in a.files:
    print(k, "bitwise equal" if np.array_equal(a[k], b[k]) else f"DIFFERS in {(a[k] != b[k]).sum()} words")
PY
rm -f $OUT/state_pf*.npz
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $OUT/pytest_gpu_r03pf.log 2>&1
RC=$?; echo "pytest rc=$RC: $(tail -1 $OUT/pytest_gpu_r03pf.log)"
[ $RC -le 1 ] || exit $RC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r03pf.log 2>&1 || exit 3
timeout -k 10 600 python bench.py > $OUT/bench_r03pf.json 2> $OUT/bench_r03pf.err || exit 4
python -c "import json;d=json.load(open('$OUT/bench_r03pf.json'));print('bench', d['value'], d['ms_per_step'], d['kernels'], d['roofline']['frac'], d['roofline']['traffic'])"
echo "chain ok"
