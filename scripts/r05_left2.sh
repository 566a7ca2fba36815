#!/usr/bin/env bash
# Round 5: the new reference-leaks GPU tests, then the leftover queue with big records (A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "leak or early_nee" > gpurun_out/pytest_gpu_leaks.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -15 gpurun_out/pytest_gpu_leaks.log
[ $rc -ne 0 ] && exit $rc
L=small-pathtracer_amd/libspt.so
ROUNDS=2 BENCH_ARGS="--config c3" timeout -k 10 400 bash scripts/ab.sh $L@SPT_LEFTOVER=0 $L@SPT_LEFT_PIECE=64 \
  "$L@SPT_LEFT_PIECE=128 SPT_LEFT_MIN=32" "$L@SPT_LEFT_PIECE=32 SPT_LEFT_MIN=48" || exit $?
cp gpurun_out/ab.txt gpurun_out/ab_c3b.txt
ROUNDS=2 BENCH_ARGS="--config c2" timeout -k 10 300 bash scripts/ab.sh $L@SPT_LEFTOVER=0 $L@SPT_LEFT_PIECE=64 \
  "$L@SPT_LEFT_PIECE=128 SPT_LEFT_MIN=32" || exit $?
cp gpurun_out/ab.txt gpurun_out/ab_c2b.txt
ROUNDS=2 BENCH_ARGS="--config c3" timeout -k 10 300 bash scripts/ab.sh "$L@SPT_LEFTOVER=0" || exit $?
timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --reference-leaks > gpurun_out/bench_refleaks.json 2>gpurun_out/bench_refleaks.err
echo "refleaks rc $?"; cat gpurun_out/bench_refleaks.json | head -c 600
