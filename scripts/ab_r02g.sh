#!/usr/bin/env bash
# A/B: where the uploaded scene's geometry is read from, per kernel level.
# Build first (CPU): scripts/build_variants.sh cur:"" sphlds:"-DSPT_SPH_LDS" slod:"-DSPT_GEO_SLOAD"
#   cur    = rect tests from the block's LDS copy, spheres by scalar loads (the default)
#   sphlds = spheres from LDS as well;  slod = rect tests by scalar loads (constant address space)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L="build/ab/cur.so build/ab/sphlds.so build/ab/slod.so"
for cfg in "c5 --spp 256" "c3 --kernel-level generic" "c3 --kernel-level cornell" "c3"; do
  BENCH_ARGS="--config $cfg" ROUNDS=2 timeout -k 10 400 bash scripts/ab.sh $L > gpurun_out/ab.txt 2>&1 || exit $?
  echo "== $cfg"; sort gpurun_out/ab.txt
done
