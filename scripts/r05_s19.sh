#!/usr/bin/env bash
# Session 19: the boxes-only-uploaded kernel for edited scenes (KV_UPBOX_NEE): the full GPU suite,
# then C3 with one box moved against the previous product (build/ab/base.so: the uploaded-geometry
# kernel), and the literal scene, 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu exit $rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for a in "--move-box 1" "--move-box -3" ""; do
    for lib in small-pathtracer_amd/libspt.so build/ab/base.so; do
      out=$(SPT_LIB=$lib timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $a 2>gpurun_out/ab_last.err) || { echo "$lib FAILED"; tail -5 gpurun_out/ab_last.err; exit 1; }
      echo "[$a] $lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["paths"]["shadow_proven_per_sample"])')"
    done
  done
done | tee gpurun_out/ab_upbox.txt
