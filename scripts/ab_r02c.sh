#!/usr/bin/env bash
# A/B: two-phase work units (phase-A units per lane, phase-B share and unit length) on C2, C3, C5@256.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
L="build/ab/steal.so build/ab/def.so build/ab/a2.so build/ab/a8.so build/ab/t06.so build/ab/t25.so build/ab/b20.so build/ab/b80.so"
for cfg in "c2" "c3" "c5 --spp 256"; do
  BENCH_ARGS="--config $cfg" ROUNDS=2 timeout -k 10 500 bash scripts/ab.sh $L > gpurun_out/ab.txt 2>&1 || exit $?
  echo "== $cfg"; sort gpurun_out/ab.txt
done
for cfg in "c2" "c3"; do
  n=$(echo $cfg | tr -d ' -'); SPT_LIB=build/ab/w_def.so SPT_WAVE_DUMP=gpurun_out/w_def_$n.bin timeout -k 10 120 $B --config $cfg > /dev/null 2>&1 || exit $?
  echo "== waves def $cfg"; python tools/wave_tail.py gpurun_out/w_def_$n.bin | tr '\n' ' '; echo
done
echo ALL_OK
