#!/usr/bin/env bash
# A/B the bench across library builds / env settings, interleaved rounds, one process per run:
#   scripts/ab.sh lib1.so lib2.so[@VAR=VALUE] ...   (ROUNDS, BENCH_ARGS from the environment)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    lib=${spec%%@*}; envs=""; [ "$spec" != "$lib" ] && envs=${spec#*@}
    out=$(env SPT_LIB=$lib $envs timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} 2>gpurun_out/ab_last.err) || { echo "$spec FAILED"; exit 1; }
    echo "$spec $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done | tee gpurun_out/ab.txt
