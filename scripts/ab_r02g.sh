#!/usr/bin/env bash
# A/B: scene geometry staged in LDS (rect tests, narrow spheres) vs scalar loads, per kernel level.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L="build/ab/cur.so build/ab/sphs.so build/ab/alls.so"
for cfg in "c5 --spp 256" "c3 --kernel-level generic" "c3 --kernel-level cornell" "c3"; do
  BENCH_ARGS="--config $cfg" ROUNDS=2 timeout -k 10 400 bash scripts/ab.sh $L > gpurun_out/ab.txt 2>&1 || exit $?
  echo "== $cfg"; sort gpurun_out/ab.txt
done
