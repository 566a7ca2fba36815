#!/usr/bin/env bash
# A/B: short-launch tuning on C2 (units per lane, stealing threshold, blocks per CU) around the
# product build (build/ab/base.so); bench.py --config c2 --steps 10 --warmup 2, 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ab() {  # lib...
  for r in 1 2 3; do
    for lib in "$@"; do
      out=$(SPT_LIB=$lib timeout -k 10 120 python bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline 2>gpurun_out/ab_last.err) || { echo "$lib FAILED"; exit 1; }
      echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
    done
  done
}
ab build/ab/base.so build/ab/su6.so build/ab/st8.so build/ab/st32.so build/ab/bpc3.so build/ab/bpc5.so | tee gpurun_out/ab_c2tune.txt
