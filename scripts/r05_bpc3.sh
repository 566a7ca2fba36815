#!/usr/bin/env bash
# A/B: resident blocks per CU x frames in flight, C3 (build/ab/bpc.so), 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=build/ab/bpc.so
for r in 1 2 3; do
  for spec in "- 2" "- 3" "SPT_BPC_CAP=4 2" "SPT_BPC_CAP=4 3" "SPT_BPC_CAP=5 2" "SPT_BPC_CAP=6 2"; do
    envs=${spec% *}; fif=${spec##* }; [ "$envs" = "-" ] && envs=""
    out=$(env SPT_LIB=$L $envs timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --frames-in-flight $fif 2>gpurun_out/ab_last.err) || { echo "$spec FAILED"; exit 1; }
    echo "$spec $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done | tee gpurun_out/ab_bpc3_c3.txt
