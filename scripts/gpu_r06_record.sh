#!/bin/bash
# Round-6 record: GPU tests, smoke, the config-2 line (CPU baseline), its
# rocprofv3 kernel summary, then configs 3, 4, 5 (bench lines; kernel
# summaries of 3 and 5).
set -o pipefail
TAG=${1:-r06r}
scripts/gpu_check_all.sh $TAG || exit 1
PROF="3 5" scripts/gpu_bench_all.sh ${TAG}_cfg 3 4 5 || exit 1
