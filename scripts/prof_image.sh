#!/usr/bin/env bash
# rocprofv3 on the image encoder microbench (tools/bench_image.py, 4096^2 synthetic): kernel trace,
# then separate PMC passes (instruction mix / stalls, LDS conflicts, HBM bytes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_img_${1:-run}
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -k 10 120 rocprofv3 "$@" --output-format csv -d $OUT/$name -o $name -- python3 tools/bench_image.py 4096 5 \
    > $OUT/$name.log 2>&1
  local rc=$?; echo "$name exit $rc"; return $rc
}
run trace --kernel-trace --stats || exit $?
run pmc1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS || exit $?
run pmc2 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE || exit $?
run pmc3 --pmc FETCH_SIZE || exit $?
run pmc4 --pmc WRITE_SIZE || exit $?
