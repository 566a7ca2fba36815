#!/usr/bin/env bash
# Session 9: young-wave cutoff A/B on C3 (SPT_YOUNG_CUT / SPT_YOUNG_RANK builds), 3 interleaved rounds,
# then C2 for the product and two cuts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ab() {  # config steps libs...
  local cfg=$1 st=$2; shift 2
  for r in 1 2 3; do
    for lib in "$@"; do
      out=$(SPT_LIB=$lib timeout -k 10 120 python bench.py --config $cfg --steps $st --warmup 2 --no-cpu-baseline 2>gpurun_out/ab_last.err) || { echo "$lib FAILED"; exit 1; }
      echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
    done
  done
}
L=build/ab
ab c3 5 $L/base.so $L/yc300r6.so $L/yc100r6.so $L/yc200r6.so $L/yc400r6.so $L/yc150r7.so $L/yc300r7.so $L/yc200r5.so $L/yc300r5.so | tee gpurun_out/ab_young_cut_c3_s9.txt
ab c2 10 $L/base.so $L/yc300r6.so $L/yc200r5.so | tee gpurun_out/ab_young_cut_c2_s9.txt
