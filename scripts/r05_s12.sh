#!/usr/bin/env bash
# Session 12: the C3 kernel levels with the final round-5 build (literal HEAD kernel, edited scene,
# the uploaded-geometry levels, reference leaks), 2 rounds, then the full GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/r05f_$tag.json \
    2> gpurun_out/r05f_$tag.err
  local rc=$?; [ $rc -eq 0 ] || { echo "bench $tag exit $rc"; tail -5 gpurun_out/r05f_$tag.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05f_$tag.json')); r=d['roofline']; print('$tag', d['value'], r['kernel_ms'], r['frac'])"
}
for i in 1 2; do
run c3_$i
run c3_movebox_$i --move-box 1
run c3_movebox_cornell_$i --move-box 1 --kernel-level cornell
run c3_cornell_$i --kernel-level cornell
run c3_const_$i --kernel-level const
run c3_generic_$i --kernel-level generic
run c3_refleaks_$i --reference-leaks
done | tee gpurun_out/r05f_levels.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu exit $rc"; tail -2 gpurun_out/pytest_gpu.log; exit $rc
