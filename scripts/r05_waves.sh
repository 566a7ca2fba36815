#!/usr/bin/env bash
# Per-wave dumps (diag build SPT_DIAG=2) of C3 and C2 with the waves' work by age rank.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in c3 c2; do
  SPT_LIB=build/ab/diag2.so timeout -k 10 200 python tools/wave_dump.py $cfg gpurun_out/waves_$cfg.bin \
    > gpurun_out/waves_$cfg.json 2> gpurun_out/waves_$cfg.err
  rc=$?; echo "$cfg exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/waves_$cfg.err; exit $rc; }
  cat gpurun_out/waves_$cfg.json
done
