#!/usr/bin/env bash
# A/B: guided-grab floor x chunk with intra-wave stealing (C2, C3), wave residency of two builds.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
for cfg in "c2 --chunk 23" "c2 --chunk 64" "c3 --chunk 48" "c3 --chunk 96" "c3 --chunk 128"; do
  BENCH_ARGS="--config $cfg" ROUNDS=1 timeout -k 10 300 bash scripts/ab.sh build/ab/steal.so build/ab/g1.so build/ab/g8.so build/ab/g16.so build/ab/g32.so > gpurun_out/ab.txt 2>&1 || exit $?
  echo "== $cfg"; cat gpurun_out/ab.txt
done
for lib in w_steal w_g16; do for cfg in "c2 --chunk 64" "c3 --chunk 96"; do
  n=$(echo $cfg | tr -d ' -'); SPT_LIB=build/ab/$lib.so SPT_WAVE_DUMP=gpurun_out/w_${lib}_$n.bin timeout -k 10 120 $B --config $cfg > /dev/null 2>&1 || exit $?
  echo "== waves $lib $cfg"; python tools/wave_tail.py gpurun_out/w_${lib}_$n.bin | tr '\n' ' '; echo
done; done
echo ALL_OK
