#!/usr/bin/env bash
# A/B the bench across library builds in one process-free loop: scripts/ab.sh lib1.so lib2.so ...
# (interleaved rounds; each run is a separate process, each prints one bench JSON line)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    out=$(SPT_LIB=$lib timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} 2>/dev/null) || { echo "$lib FAILED"; exit 1; }
    echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done | tee gpurun_out/ab.txt
