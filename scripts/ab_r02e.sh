#!/usr/bin/env bash
# A/B: in-wave stealing + small-launch unit policy; then the GPU parity suite.
# Build first (CPU): scripts/build_variants.sh cur:"" nosteal:"-DSPT_NO_STEAL" \
#   su1:"-DSPT_SMALL_UNITS=1.0" su2:"-DSPT_SMALL_UNITS=2.0" su3:"-DSPT_SMALL_UNITS=3.0"
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L="build/ab/cur.so build/ab/nosteal.so build/ab/su1.so build/ab/su2.so build/ab/su3.so"
for cfg in "c2" "c3" "c5 --spp 256" "c4 --spp 128"; do
  BENCH_ARGS="--config $cfg" ROUNDS=2 timeout -k 10 500 bash scripts/ab.sh $L > gpurun_out/ab.txt 2>&1 || exit $?
  echo "== $cfg"; sort gpurun_out/ab.txt
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest $rc"; tail -3 gpurun_out/pytest_gpu.log; exit $rc
