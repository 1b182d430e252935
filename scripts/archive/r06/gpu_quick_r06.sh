#!/bin/bash
set -o pipefail
O=gpurun_out/r06a; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/b2.json 2> $O/b2.err || { tail -5 $O/b2.err; exit 1; }
cut -c1-400 $O/b2.json
timeout -k 10 300 python bench.py --config 3 --steps 50 --warmup 5 --no-cpu-baseline > $O/b3.json 2> $O/b3.err || { tail -5 $O/b3.err; exit 1; }
cut -c1-400 $O/b3.json
