#!/usr/bin/env bash
# A/B: resident blocks per CU for the short C2 launch (build/ab/bpc.so), 4 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=build/ab/bpc.so
ROUNDS=4 BENCH_ARGS="--config c2 --steps 10" timeout -k 10 600 bash scripts/ab.sh $L $L@SPT_BPC_CAP=6 $L@SPT_BPC_CAP=4 || exit $?
cp gpurun_out/ab.txt gpurun_out/ab_bpc2_c2.txt
