#!/usr/bin/env bash
# Session 21: the boxes-only-uploaded cosine kernel (KV_UPBOX_COS): the full GPU suite, then C2 with
# one box moved against the previous product (build/ab/base.so: KV_CORNELL_COS), 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu exit $rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for a in "--config c2 --move-box 1" "--config c2"; do
    for lib in small-pathtracer_amd/libspt.so build/ab/base.so; do
      out=$(SPT_LIB=$lib timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $a 2>gpurun_out/ab_last.err) || { echo "$lib FAILED"; tail -5 gpurun_out/ab_last.err; exit 1; }
      echo "[$a] $lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
    done
  done
done | tee gpurun_out/ab_upbox_cos.txt
