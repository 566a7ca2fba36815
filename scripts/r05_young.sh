#!/usr/bin/env bash
# Round 5: the young waves' queue -- parity on C3 rows, then A/B on C3 / C2 / C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "young" > gpurun_out/pytest_young.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_young.log; [ $rc -eq 0 ] || exit $rc
L=small-pathtracer_amd/libspt.so
ROUNDS=2 BENCH_ARGS="--config c3" timeout -k 10 600 bash scripts/ab.sh $L $L@SPT_YOUNG_PCT=10 $L@SPT_YOUNG_PCT=20 $L@SPT_YOUNG_PCT=30 \
  "$L@SPT_YOUNG_PCT=20 SPT_YOUNG_CHUNK=48" "$L@SPT_YOUNG_PCT=20 SPT_YOUNG_RANK=5" "$L@SPT_YOUNG_PCT=20 SPT_YOUNG_CHUNK=12" || exit $?
cp gpurun_out/ab.txt gpurun_out/ab_young_c3.txt
