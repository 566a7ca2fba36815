#!/usr/bin/env bash
# PMC passes (one counter group per run) on the encoder microbench (tools/bench_image.py 4096^2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out gpurun_out/enc_pmc
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/enc_pmc/p$i -o p$i \
    -- python3 tools/bench_image.py 4096 3 > gpurun_out/enc_pmc/p$i.log 2>&1
  rc=$?; echo "pass $i exit $rc"; [ $rc -eq 0 ] || exit $rc
done
