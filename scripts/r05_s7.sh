#!/usr/bin/env bash
# Round 5 session 7: GPU tests, then C2 / C3 with short launches at 4 blocks per CU (default now).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu exit $rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for cfg in c2 c3; do
    timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05_s7_${cfg}_$i.json 2>gpurun_out/r05_s7.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/r05_s7_${cfg}_$i.json')); r=d['roofline']; print('$cfg', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'])"
  done
done
