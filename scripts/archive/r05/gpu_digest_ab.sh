#!/bin/bash
# Bitwise digests of two libraries at the bench shape, then an interleaved A/B.
#   usage: scripts/gpu_digest_ab.sh TAG var_a var_b
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for V in "$@"; do
  HN_LIB_PATH=hashnerf-pytorch_amd/build/$V.so timeout -k 10 200 python scripts/variant_digest.py > $O/digest_$V.txt 2>&1 \
      || { tail -5 $O/digest_$V.txt; exit 1; }
  echo "$V $(tail -1 $O/digest_$V.txt)"
done
REPS=${REPS:-1} scripts/gpu_ab_var.sh $TAG "$@"
