#!/usr/bin/env bash
# rocprofv3 passes on the bench workload (kernel trace + separate PMC passes; never combined with
# sys/runtime traces). Output under gpurun_out/prof_<tag>/. Usage: scripts/profile.sh TAG [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift || true
# one frame in flight: every render dispatch runs alone, so the trace's average duration is the
# isolated kernel time the bench line's roofline.kernel_ms reports (two overlapping frames stretch
# each other's dispatch spans)
# --no-extras: no render launches after the timed region (reference-leaks leg, quality renders), so
# the --stats summary's average is the warm-up and timed dispatches of the one kernel
ARGS=${*:---steps 20 --warmup 3 --no-cpu-baseline --frames-in-flight 1 --no-extras}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" --output-format csv -d $OUT/$name -o $name -- python3 bench.py $ARGS \
    > $OUT/$name.log 2>&1
  local rc=$?; echo "$name exit $rc"; return $rc
}
run trace --kernel-trace --stats || exit $?
run pmc1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM || exit $?
run pmc2 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE || exit $?
run pmc3 --pmc FETCH_SIZE || exit $?
run pmc4 --pmc WRITE_SIZE || exit $?
find $OUT -name "*.csv" | head -20
