#!/usr/bin/env bash
# Session 8: C2 short-launch tuning (scripts/r05_c2tune.sh), then the young-wave cutoff A/B on C3
# (SPT_YOUNG_CUT / SPT_YOUNG_RANK builds against the product build), 3 interleaved rounds each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 bash scripts/r05_c2tune.sh || exit $?
for r in 1 2 3; do
  for lib in build/ab/base.so build/ab/yc500.so build/ab/yc700.so build/ab/yc850.so build/ab/yc700r6.so build/ab/yc300r6.so; do
    out=$(SPT_LIB=$lib timeout -k 10 120 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline 2>gpurun_out/ab_last.err) || { echo "$lib FAILED"; exit 1; }
    echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done | tee gpurun_out/ab_young_cut_c3.txt
