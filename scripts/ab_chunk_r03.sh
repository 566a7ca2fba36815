#!/usr/bin/env bash
# Round-3 unit-size re-check with the unit slots (a unit's retire is now plain stores): the C3 bench
# line first (cool GPU), then interleaved A/B of SPT_CHUNK on C3 and C2 (scripts/ab.sh, in-tree library).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=small-pathtracer_amd/libspt.so
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/r03_bench_c3.json 2> gpurun_out/r03_bench_c3.err
rc=$?; echo "bench c3 exit $rc"; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash scripts/ab.sh $L@SPT_CHUNK=0 $L@SPT_CHUNK=32 $L@SPT_CHUNK=40 $L@SPT_CHUNK=64 > gpurun_out/ab_chunk_c3.txt || exit $?
BENCH_ARGS="--config c2" ROUNDS=3 bash scripts/ab.sh $L@SPT_CHUNK=0 $L@SPT_CHUNK=32 $L@SPT_CHUNK=22 > gpurun_out/ab_chunk_c2.txt || exit $?
cat gpurun_out/ab_chunk_c3.txt gpurun_out/ab_chunk_c2.txt
