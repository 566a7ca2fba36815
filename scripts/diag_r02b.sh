#!/usr/bin/env bash
# C2 after stealing: wave residency, VALU per iteration (PMC), and the C3 bench with the new quality fixture.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
for cfg in c2 c3; do
  SPT_LIB=build/ab/waves.so SPT_WAVE_DUMP=gpurun_out/wv_$cfg.bin timeout -k 10 120 $B --config $cfg > gpurun_out/wv_$cfg.log 2>&1 || exit $?
  echo "== waves $cfg"; python3 tools/wave_tail.py gpurun_out/wv_$cfg.bin | tr '\n' ' '; echo
done
OUT=gpurun_out/pmc_c2; mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 --output-format csv -d $OUT/p1 -o p1 -- $B --config c2 > $OUT/p1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o p2 -- $B --config c2 > $OUT/p2.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o tr -- $B --config c2 > $OUT/tr.log 2>&1 || exit $?
python3 scripts/pmc_summary.py $OUT > $OUT/summary.json; python3 -c "import json; d=json.load(open('$OUT/summary.json')); print(json.dumps(d['counters'])); print(json.dumps(d['derived']))"
timeout -k 10 120 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_q.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/bench_q.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_ms'], json.dumps(d['quality']))"
