#!/usr/bin/env bash
# Round 5: GPU parity tests with the leftover launch, then A/B of the leftover queue on C3 and C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu exit $rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
L=small-pathtracer_amd/libspt.so
ROUNDS=3 BENCH_ARGS="--config c3" timeout -k 10 400 bash scripts/ab.sh $L@SPT_LEFTOVER=0 $L@SPT_LEFTOVER=1 \
  $L@SPT_LEFT_PIECE=8 $L@SPT_LEFT_PIECE=32 || exit $?
cp gpurun_out/ab.txt gpurun_out/ab_c3.txt
ROUNDS=3 BENCH_ARGS="--config c2" timeout -k 10 300 bash scripts/ab.sh $L@SPT_LEFTOVER=0 $L@SPT_LEFTOVER=1 \
  $L@SPT_LEFT_PIECE=8 $L@SPT_LEFT_PIECE=32 || exit $?
cp gpurun_out/ab.txt gpurun_out/ab_c2.txt
