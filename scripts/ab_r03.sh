#!/usr/bin/env bash
# Round-3 A/B session: GPU tests on the in-tree build, interleaved timing rounds of library
# variants (scripts/ab.sh), then one WRITE_SIZE pass per variant (memory-side atomic traffic).
#   scripts/ab_r03.sh lib1.so lib2.so ...   (ROUNDS, BENCH_ARGS, NO_TESTS from the environment)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest -m gpu exit $rc"; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
ROUNDS=${ROUNDS:-3} bash scripts/ab.sh "$@" || exit $?
if [ -n "${PMC:-}" ]; then
  for lib in "$@"; do
    name=$(basename $lib .so)
    SPT_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/ws_$name -o ws \
      -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ws_$name.log 2>&1
    rc=$?; echo "$name WRITE_SIZE pass exit $rc"; [ $rc -eq 0 ] || exit $rc
  done
fi
