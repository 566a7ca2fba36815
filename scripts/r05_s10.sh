#!/usr/bin/env bash
# Session 10: the young-block cut in the product build: GPU tests, then A/B against the previous
# product (build/ab/base.so) on C3 (3 rounds), C4 and C5 (A/B sizes, 2 rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu exit $rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
ab() {  # rounds args libs...
  local n=$1 args=$2; shift 2
  for r in $(seq 1 $n); do
    for lib in "$@"; do
      out=$(SPT_LIB=$lib timeout -k 10 200 python bench.py $args --no-cpu-baseline 2>gpurun_out/ab_last.err) || { echo "$lib FAILED"; exit 1; }
      echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
    done
  done
}
N=small-pathtracer_amd/libspt.so B=build/ab/base.so
ab 3 "--config c3 --steps 5 --warmup 2" $B $N | tee gpurun_out/ab_s10_c3.txt
ab 2 "--config c4 --steps 2 --warmup 1" $B $N | tee gpurun_out/ab_s10_c4.txt
ab 2 "--config c5 --spp 256 --steps 2 --warmup 1" $B $N | tee gpurun_out/ab_s10_c5.txt
