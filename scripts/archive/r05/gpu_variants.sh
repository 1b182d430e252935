#!/bin/bash
# Variant libraries (hashnerf-pytorch_amd/build/<name>.so): bitwise digests of
# one bench-shape forward + backward, then interleaved short bench lines and
# (PROF=1) rocprof kernel stats -- scripts/gpu_lib_ab.sh.
#   usage: REPS=2 PROF=1 scripts/gpu_variants.sh TAG var_a var_b ...
set -o pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for V in "${@:2}"; do
  HN_LIB_PATH=hashnerf-pytorch_amd/build/$V.so timeout -k 10 200 python scripts/variant_digest.py $DIGEST_ARGS \
      > $OUT/digest_$V.txt 2>&1 || { tail -5 $OUT/digest_$V.txt; exit 1; }
  echo "$V $(tail -1 $OUT/digest_$V.txt)"
done
scripts/gpu_lib_ab.sh "$@"
