#!/usr/bin/env bash
# Session 23: the young-block cut on the sphere NEE kernel (C5 at the A/B size, 4096^2 @ 256 spp) at
# other cut points / ranks (build/ab/sph_c<cut>_r<rank>.so) against the product (no cut there),
# 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=build/ab
for r in 1 2 3; do
  for lib in small-pathtracer_amd/libspt.so $L/sph_c300_r6.so $L/sph_c700_r6.so $L/sph_c850_r6.so $L/sph_c300_r7.so; do
    out=$(SPT_LIB=$lib timeout -k 10 150 python bench.py --config c5 --spp 256 --steps 2 --warmup 1 --no-cpu-baseline 2>gpurun_out/ab_last.err) || { echo "$lib FAILED"; exit 1; }
    echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done | tee gpurun_out/ab_sph_cut.txt
