#!/usr/bin/env bash
# A/B library builds on C3, C2 and C5 (256 spp) in interleaved rounds, one bench process per run:
#   scripts/ab_configs.sh lib1.so lib2.so ...   (ROUNDS from the environment, default 2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 $ROUNDS); do
  for cfg in "c3" "c2" "c5 --spp 256"; do
    for lib in "$@"; do
      out=$(SPT_LIB=$lib timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --config $cfg 2>gpurun_out/ab_last.err) || { echo "$lib $cfg FAILED"; exit 1; }
      echo "$lib ${cfg%% *} $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
    done
  done
done | tee gpurun_out/ab_configs.txt
