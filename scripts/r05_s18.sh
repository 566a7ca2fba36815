#!/usr/bin/env bash
# Session 18: bench.py --gpus N spawning its own ranks with the final round-5 build (gloo rehearsal
# on the one GPU: ranks share the device, the gather goes through host memory; rank 0 re-renders the
# whole image alone and compares), N = 2, 4, 8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 2 4 8; do
  timeout -k 10 400 env SPT_DIST_BACKEND=gloo python bench.py --gpus $n --steps 3 --warmup 1 \
    --no-cpu-baseline > gpurun_out/spawnf$n.json 2> gpurun_out/spawnf$n.err
  rc=$?; echo "spawn $n exit $rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/spawnf$n.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/spawnf$n.json')); print($n, d['n_gpus'], d['value'], d['config']['spp'], d['gather_equals_1gpu_render'], d['ranks']['kernel_ms'])"
done
