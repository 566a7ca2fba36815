#!/usr/bin/env bash
# Session 11: units per resident lane of a long launch (SPT_UNITS_PER_LANE 4 / 6 / 8 = product / 12:
# C3 chunks 192 / 128 / 96 / 64 samples) with the young-block cut in place; C3, 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=build/ab
for r in 1 2 3; do
  for lib in $L/base.so $L/upl4.0.so $L/upl6.0.so $L/upl12.0.so; do
    out=$(SPT_LIB=$lib timeout -k 10 120 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline 2>gpurun_out/ab_last.err) || { echo "$lib FAILED"; exit 1; }
    echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done | tee gpurun_out/ab_upl_c3.txt
