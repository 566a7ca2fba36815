#!/usr/bin/env bash
# Unit size vs bench value and isolated kernel time, interleaved rounds (no PMC passes):
#   scripts/ab_chunk_times.sh CHUNK...   (0 = auto; ROUNDS, CFG from the environment)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for c in "$@"; do
    out=$(timeout -k 10 120 python bench.py --config ${CFG:-c3} --steps 8 --warmup 2 --no-cpu-baseline --chunk $c 2>/dev/null) || { echo "chunk $c FAILED"; exit 1; }
    echo "chunk $c $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
  done
done | tee gpurun_out/ab_chunk_times.txt
