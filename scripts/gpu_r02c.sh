#!/usr/bin/env bash
# Round-2 measurement refresh: default bench (CPU baselines + quality), C2/C4/C5 lines, rocprofv3
# kernel trace + PMC passes of C3 (scripts/profile.sh r02).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name exit $rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300
  return $rc
}
step bench 400 python -u bench.py || exit $?
step bench_c2 120 python -u bench.py --config c2 --steps 5 --warmup 1 --no-cpu-baseline || exit $?
step bench_c4 200 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline || exit $?
step bench_c5 200 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline || exit $?
step profile 600 bash scripts/profile.sh ${PROF_TAG:-r02} || exit $?
echo ALL_OK
