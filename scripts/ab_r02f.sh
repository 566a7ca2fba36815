#!/usr/bin/env bash
# A/B for DESIGN section 4: the HEAD-topology kernel reading its rect tests by scalar loads (s_load,
# constant address space), from an LDS copy (-DSPT_GEO_LDS), or as instruction literals (auto).
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
BENCH_ARGS="--config c3 --kernel-level cornell" ROUNDS=2 timeout -k 10 300 bash scripts/ab.sh build/ab/cur.so build/ab/lds.so > gpurun_out/ab_geo.txt 2>&1 || exit $?
BENCH_ARGS="--config c3 --kernel-level generic" ROUNDS=2 timeout -k 10 300 bash scripts/ab.sh build/ab/cur.so build/ab/lds.so > gpurun_out/ab_geo_gen.txt 2>&1 || exit $?
BENCH_ARGS="--config c3" ROUNDS=2 timeout -k 10 300 bash scripts/ab.sh build/ab/cur.so > gpurun_out/ab_geo_auto.txt 2>&1 || exit $?
echo "== cornell (s_load vs LDS)"; cat gpurun_out/ab_geo.txt; echo "== generic"; cat gpurun_out/ab_geo_gen.txt; echo "== auto (literals)"; cat gpurun_out/ab_geo_auto.txt
