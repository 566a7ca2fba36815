#!/usr/bin/env bash
# Round-3 diagnostic session (C2 tail / unit size): region statistics (-DSPT_DIAG=1) and per-wave
# residency (-DSPT_DIAG=2) at C2's auto unit (64 samples) and 32 samples, and C3, one render each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # lib tag args...
  local lib=$1 tag=$2; shift 2
  SPT_LIB=$lib SPT_WAVE_DUMP=gpurun_out/waves_$tag.bin timeout -k 10 120 python bench.py --steps 1 --warmup 0 \
    --no-cpu-baseline "$@" > gpurun_out/diag_$tag.json 2> gpurun_out/diag_$tag.err
  local rc=$?; echo "$tag exit $rc"; return $rc
}
run build/ab/diag1.so rs_c2_64 --config c2 || exit $?
run build/ab/diag1.so rs_c2_32 --config c2 --chunk 32 || exit $?
run build/ab/diag1.so rs_c3 || exit $?
run build/ab/diag2.so wt_c2_64 --config c2 || exit $?
run build/ab/diag2.so wt_c2_32 --config c2 --chunk 32 || exit $?
run build/ab/diag2.so wt_c3 || exit $?
