#!/usr/bin/env bash
# A/B: resident blocks per CU (SPT_BPC_CAP, build/ab/bpc.so), C3 and C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=build/ab/bpc.so
ROUNDS=2 BENCH_ARGS="--config c3" timeout -k 10 500 bash scripts/ab.sh $L $L@SPT_BPC_CAP=7 $L@SPT_BPC_CAP=6 $L@SPT_BPC_CAP=5 $L@SPT_BPC_CAP=4 || exit $?
cp gpurun_out/ab.txt gpurun_out/ab_bpc_c3.txt
ROUNDS=2 BENCH_ARGS="--config c2" timeout -k 10 400 bash scripts/ab.sh $L $L@SPT_BPC_CAP=7 $L@SPT_BPC_CAP=6 $L@SPT_BPC_CAP=5 $L@SPT_BPC_CAP=4 || exit $?
cp gpurun_out/ab.txt gpurun_out/ab_bpc_c2.txt
