#!/usr/bin/env bash
# Extra PMC passes on C3 (stall and instruction-class counters), one pass per group, each bounded.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcx; mkdir -p $OUT
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
i=0
for grp in "SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_IFETCH SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FLOPS_FP32" \
           "SQ_ACTIVE_INST_VALU2 SQ_INSTS_VSKIPPED SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS" \
           "SQC_ICACHE_MISSES SQC_ICACHE_HITS" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o p$i -- $B > $OUT/p$i.log 2>&1; rc=$?
  echo "pass $i exit $rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_summary.py $OUT > $OUT/summary.json; cat $OUT/summary.json
