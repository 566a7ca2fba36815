#!/usr/bin/env bash
# Marginal issue cost of 24 extra SALU / VALU per wave-iteration (diagnostic builds SPT_DIAG=3/4).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=3 BENCH_ARGS="--config c3 --frames-in-flight 1" timeout -k 10 600 bash scripts/ab.sh \
  small-pathtracer_amd/libspt.so build/ab/diag3.so build/ab/diag4.so || exit $?
cp gpurun_out/ab.txt gpurun_out/ab_probe.txt
