#!/usr/bin/env bash
# Frames in flight (bench.py --frames-in-flight, FIFS = the values to interleave, default "1 2 1 2") on
# C3 and C2 (CFGS), then the 2/4-rank gloo rehearsals (REHEARSAL=0 skips them).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
show() { python3 -c "import json,sys; d=json.load(open('gpurun_out/fif.json')); r=d['roofline']; print(sys.argv[1], d['config']['frames_in_flight'], d['value'], d['ms_per_step'], r['kernel_ms'], r['kernel_ms_in_flight'], r['frac'], r['frac_pipelined'], (d.get('quality') or {}).get('rmse_vs_contract'))" $1; }
for cfg in ${CFGS:-c3 c2}; do
  st=10; [ $cfg = c2 ] && st=20
  for a in ${FIFS:-1 2 1 2}; do
    timeout -k 10 200 python bench.py --config $cfg --steps $st --warmup 2 --no-cpu-baseline --frames-in-flight $a \
      > gpurun_out/fif.json 2> gpurun_out/fif.err || exit $?
    show $cfg
  done
done
[ "${REHEARSAL:-1}" = 0 ] || RANKS="2 4" bash scripts/rehearsal_r02.sh
