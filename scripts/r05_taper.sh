#!/usr/bin/env bash
# A/B: tapered last passes (SPT_TAPER, build/ab/taper*.so) against the product build (build/ab/base.so),
# C3; GPU parity suite on the taper build first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SPT_LIB=build/ab/taper8.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/taper_parity.log 2>&1
rc=$?; echo "parity (taper8) exit $rc"; tail -2 gpurun_out/taper_parity.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 BENCH_ARGS="--config c3" timeout -k 10 700 bash scripts/ab.sh build/ab/base.so build/ab/taper8.so build/ab/taper16.so build/ab/taper4.so build/ab/taper8u4.so || exit $?
cp gpurun_out/ab.txt gpurun_out/ab_taper_c3.txt
