#!/usr/bin/env bash
# A/B: guided grabs and intra-wave sample stealing (C2, C3), then the GPU parity suite on the new
# default build.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
BENCH_ARGS="--config c2" ROUNDS=2 timeout -k 10 300 bash scripts/ab.sh build/ab/base.so build/ab/guided.so build/ab/steal.so build/ab/both.so > gpurun_out/ab_c2.txt 2>&1 || exit $?
BENCH_ARGS="--config c3" ROUNDS=2 timeout -k 10 300 bash scripts/ab.sh build/ab/base.so build/ab/guided.so build/ab/steal.so build/ab/both.so > gpurun_out/ab_c3.txt 2>&1 || exit $?
for ch in 32 64; do BENCH_ARGS="--config c2 --chunk $ch" ROUNDS=1 timeout -k 10 120 bash scripts/ab.sh build/ab/both.so > gpurun_out/ab_c2_ch$ch.txt 2>&1 || exit $?; done
for ch in 64 96 128; do BENCH_ARGS="--config c3 --chunk $ch" ROUNDS=1 timeout -k 10 120 bash scripts/ab.sh build/ab/both.so > gpurun_out/ab_c3_ch$ch.txt 2>&1 || exit $?; done
cat gpurun_out/ab_c2.txt gpurun_out/ab_c3.txt gpurun_out/ab_c2_ch*.txt gpurun_out/ab_c3_ch*.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
