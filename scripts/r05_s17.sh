#!/usr/bin/env bash
# Session 17: the last pass on a counter of its own, taken first by the young blocks (SPT_YQ builds
# build/ab/yq_c<cut>_r<rank>.so) against the product (build/ab/base.so); the full-size parity tests
# on one YQ build first; C3, 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SPT_LIB=build/ab/yq_c1000_r4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "full_size" > gpurun_out/yq_parity.log 2>&1
rc=$?; echo "parity (yq) exit $rc"; tail -2 gpurun_out/yq_parity.log; [ $rc -eq 0 ] || exit $rc
L=build/ab
for r in 1 2 3; do
  for lib in $L/base.so $L/yq_c300_r6.so $L/yq_c1000_r6.so $L/yq_c1000_r5.so $L/yq_c1000_r4.so $L/yq_c300_r4.so; do
    out=$(SPT_LIB=$lib timeout -k 10 120 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline 2>gpurun_out/ab_last.err) || { echo "$lib FAILED"; exit 1; }
    echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done | tee gpurun_out/ab_yq_c3.txt
