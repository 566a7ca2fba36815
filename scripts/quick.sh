#!/usr/bin/env bash
# Iteration run on the GPU box: GPU parity tests, then the C3 bench without the CPU baseline.
# Usage: scripts/quick.sh [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu exit $rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${*} > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
rc2=$?; echo "bench exit $rc2"; cat gpurun_out/bench_quick.json; tail -3 gpurun_out/bench_quick.err
exit $(( rc != 0 ? rc : rc2 ))
