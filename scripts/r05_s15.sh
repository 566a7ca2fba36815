#!/usr/bin/env bash
# Session 15: guided grabs in long launches (SPT_GUIDED_LONG = shift offset; build/ab/gl*.so) against
# the product (build/ab/base.so), C3, 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=build/ab
for r in 1 2 3; do
  for lib in $L/base.so $L/gl0.so $L/gl-2.so $L/gl-4.so $L/gl2.so; do
    out=$(SPT_LIB=$lib timeout -k 10 120 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline 2>gpurun_out/ab_last.err) || { echo "$lib FAILED"; exit 1; }
    echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done | tee gpurun_out/ab_guided_long_c3.txt
