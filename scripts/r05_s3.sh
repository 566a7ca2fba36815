#!/usr/bin/env bash
# Round 5 session 3: bench.py --gpus N spawning its own ranks (gloo rehearsal on the one GPU), and
# the leftover launch's two dispatches under rocprofv3 (C3, C2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 2 4; do
  timeout -k 10 300 env SPT_DIST_BACKEND=gloo python bench.py --gpus $n --steps 3 --warmup 1 \
    --no-cpu-baseline > gpurun_out/spawn$n.json 2> gpurun_out/spawn$n.err
  rc=$?; echo "spawn $n exit $rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/spawn$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/spawn$n.json')); print($n, d['n_gpus'], d['value'], d['config']['spp'], d['gather_equals_1gpu_render'], d['ranks'])"
done
for cfg in c3 c2; do
  OUT=gpurun_out/prof_left_$cfg; mkdir -p $OUT
  SPT_LEFTOVER=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o left -- \
    python3 bench.py --config $cfg --steps 4 --warmup 1 --no-cpu-baseline --frames-in-flight 1 > $OUT/log 2>&1
  echo "rocprof $cfg exit $?"
done
find gpurun_out/prof_left_* -name "*kernel_stats.csv" | xargs -I{} sh -c 'echo {}; cat {}'
