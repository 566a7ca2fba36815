#!/usr/bin/env bash
# Per-wave dumps of C3 with and without the young-block cut (diag builds, tools/wave_dump.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SPT_LIB=build/ab/diag2.so timeout -k 10 180 python tools/wave_dump.py c3 gpurun_out/waves_c3_cut.bin > gpurun_out/waves_c3_cut.json || exit $?
SPT_LIB=build/ab/diag2_nocut.so timeout -k 10 180 python tools/wave_dump.py c3 gpurun_out/waves_c3_nocut.bin > gpurun_out/waves_c3_nocut.json || exit $?
rm -f gpurun_out/waves_c3_*.bin
