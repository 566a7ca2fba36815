#!/usr/bin/env bash
# Session 13: the young-block cut on the other rect kernels (edited scene, uploaded geometry, the
# const and reference-leaks levels): product (libspt.so) against SPT_YOUNG_CUT=0 (build/ab/nocut.so), 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for a in "--move-box 1" "--move-box 1 --kernel-level cornell" "--kernel-level const" "--reference-leaks"; do
    for lib in small-pathtracer_amd/libspt.so build/ab/nocut.so; do
      out=$(SPT_LIB=$lib timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $a 2>gpurun_out/ab_last.err) || { echo "$lib FAILED"; exit 1; }
      echo "$(echo $a | tr -d ' -') $lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
    done
  done
done | tee gpurun_out/ab_s13_levels.txt
