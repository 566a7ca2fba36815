#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel stats. Stops at the first GPU
# fault/abort/timeout (exit codes other than 0/1 from pytest).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/gpu_info.txt 2>&1 || true
timeout -k 10 90 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke0.log 2>&1 || { echo "pre-smoke failed $?"; cat gpurun_out/smoke0.log | tail -5; exit 3; }
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest -m gpu exit $rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
exit $rc
