#!/usr/bin/env bash
# Session 20: the young-block cut on the boxes-only-uploaded kernel (build/ab/upcut.so) against the
# product (no cut there), C3 with one box moved, 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for lib in small-pathtracer_amd/libspt.so build/ab/upcut.so; do
    out=$(SPT_LIB=$lib timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --move-box 1 2>gpurun_out/ab_last.err) || { echo "$lib FAILED"; exit 1; }
    echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done | tee gpurun_out/ab_upcut.txt
