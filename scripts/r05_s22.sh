#!/usr/bin/env bash
# Session 22: young waves past the cut raise their SIMD priority (s_setprio SPT_YOUNG_PRIO; builds
# build/ab/yp*.so, yp3c700/850 = cut at 70 / 85 %) against the product, C3, 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=build/ab
for r in 1 2 3; do
  for lib in small-pathtracer_amd/libspt.so $L/yp3.so $L/yp1.so $L/yp3c700.so $L/yp3c850.so; do
    out=$(SPT_LIB=$lib timeout -k 10 120 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline 2>gpurun_out/ab_last.err) || { echo "$lib FAILED"; exit 1; }
    echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done | tee gpurun_out/ab_young_prio.txt
