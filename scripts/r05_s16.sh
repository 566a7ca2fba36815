#!/usr/bin/env bash
# Session 16: with the young-block cut in place, the pixel-order spreading factor (SPT_SCRAMBLE_K
# 1 / 8 = product / 32 / 256) and the stealing threshold of long launches (SPT_STEAL_MIN 4 / 8 =
# product / 16); C3, 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=build/ab
for r in 1 2 3; do
  for lib in $L/base.so $L/sk1.so $L/sk32.so $L/sk256.so $L/sm4.so $L/sm16.so; do
    out=$(SPT_LIB=$lib timeout -k 10 120 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline 2>gpurun_out/ab_last.err) || { echo "$lib FAILED"; exit 1; }
    echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done | tee gpurun_out/ab_s16_c3.txt
