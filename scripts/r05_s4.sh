#!/usr/bin/env bash
# Round 5 session 4: all GPU tests, then the bench lines this round adds: C3 with the reference's
# leaked paths, C3 on an edited rect[] (short box moved 1 in x: the uploaded-geometry kernels) and
# C3 capped at each kernel level, C2 with its full-size quality leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu exit $rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, env assignments ("-" for none), bench args...
  local tag=$1 envs=$2; shift 2; [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/r05_$tag.json \
    2> gpurun_out/r05_$tag.err
  local rc=$?; echo "bench $tag exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r05_$tag.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05_$tag.json')); r=d['roofline']; print('$tag', d['value'], r['kernel_ms'], r['frac'])"
}
run c3 -
run c3_side16 SPT_SIDE=16
run c3_side32 SPT_SIDE=32
run c3_side16_c16 "SPT_SIDE=16 SPT_SIDE_CHUNK=16"
run c3_1fly - --frames-in-flight 1
run c3_side16_1fly SPT_SIDE=16 --frames-in-flight 1
run c2 - --config c2
run c2_side8 SPT_SIDE=8 --config c2
run c2_side16 SPT_SIDE=16 --config c2
run c3_refleaks - --reference-leaks
run c3_movebox - --move-box 1
run c3_movebox_cornell - --move-box 1 --kernel-level cornell
run c3_cornell - --kernel-level cornell
run c3_const - --kernel-level const
run c3_generic - --kernel-level generic
