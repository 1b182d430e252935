#!/bin/bash
# Round-5 PMC traffic for configs 2, 3 and 5 (the files bench.py reads).
set -o pipefail
bash scripts/gpu_pmc.sh r05c2 || exit 1
bash scripts/gpu_pmc.sh r05c3 --config 3 || exit 1
bash scripts/gpu_pmc.sh r05c5 --config 5 || exit 1
ls -la gpurun_out/traffic_r05c*.json
