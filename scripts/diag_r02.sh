#!/usr/bin/env bash
# Round-2 diagnostics: C2 queue tail (per-wave times, region stats), C2 chunk sweep, C2/C3 PMC.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
run() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name exit $rc"; tail -2 gpurun_out/$name.log; return $rc; }
run waves_c2 120 env SPT_LIB=build/ab/waves.so SPT_WAVE_DUMP=gpurun_out/waves_c2.bin $B --config c2 || exit $?
run waves_c3 120 env SPT_LIB=build/ab/waves.so SPT_WAVE_DUMP=gpurun_out/waves_c3.bin $B --config c3 || exit $?
run regions_c2 120 env SPT_LIB=build/ab/regions.so $B --config c2 || exit $?
run regions_c3 120 env SPT_LIB=build/ab/regions.so $B --config c3 || exit $?
for ch in 8 12 16 23 32 64; do run chunk_c2_$ch 120 $B --config c2 --chunk $ch || exit $?; done
for ch in 24 48 96; do run chunk_c3_$ch 120 $B --config c3 --chunk $ch || exit $?; done
python tools/wave_tail.py gpurun_out/waves_c2.bin
python tools/wave_tail.py gpurun_out/waves_c3.bin
grep -h SPT_REGION gpurun_out/regions_c*.log
echo ALL_OK
