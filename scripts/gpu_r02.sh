#!/usr/bin/env bash
# Round-2 GPU session: smoke, the -m gpu suite, the default bench (with its CPU baselines), the
# drop-in program on 1 device through the multi-GPU entry point, and the classic-box diagnostic.
# Every GPU step has its own time limit; the session stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name exit $rc"; tail -4 "gpurun_out/$name.log"
  return $rc
}
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread || exit $?
step bench 400 python -u bench.py || exit $?
step devices1 120 small-pathtracer_amd/smallpt_amd 1024 768 64 1 gpurun_out/dev1.ppm --devices 1 || exit $?
step classic_anchor 200 python -u tools/classic_anchor.py --spp 1024 || exit $?
echo ALL_OK
