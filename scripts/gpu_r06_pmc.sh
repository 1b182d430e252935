#!/bin/bash
# Round-6 PMC traffic files for bench.py's roofline.traffic: configs 2, 3, 5
# (one rocprofv3 pass per counter group, scripts/gpu_pmc.sh), copied to
# gpurun_out/<tag>/traffic_config<N>_procedural_p1000_binned.json.
set -o pipefail
TAG=${1:-r06p}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
for C in ${CFGS:-2 3 5}; do
  timeout -k 10 900 scripts/gpu_pmc.sh ${TAG}c$C --config $C > $O/pmc_c$C.log 2>&1 || { tail -5 $O/pmc_c$C.log; exit 1; }
  cp gpurun_out/traffic_${TAG}c$C.json $O/traffic_config${C}_procedural_p1000_binned.json
  cp gpurun_out/pmc_${TAG}c$C.txt $O/
  python3 -c "import json;t=json.load(open('$O/traffic_config${C}_procedural_p1000_binned.json'));ks=t['kernels'];print('config $C', {k: round((v.get('fetch_bytes',0)+v.get('write_bytes',0))/1e6,1) for k,v in ks.items()})"
done
