#!/usr/bin/env bash
# A/B working tree (new) vs HEAD (old) on C5@256 and C3, then the GPU parity suite.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for cfg in "c5 --spp 256" "c3"; do
  BENCH_ARGS="--config $cfg" ROUNDS=2 timeout -k 10 400 bash scripts/ab.sh build/ab/old.so build/ab/new.so > gpurun_out/ab.txt 2>&1 || exit $?
  echo "== $cfg"; sort gpurun_out/ab.txt
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest $rc"; tail -3 gpurun_out/pytest_gpu.log; exit $rc
