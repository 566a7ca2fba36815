#!/usr/bin/env bash
# Round 5 session 6: the edited-geometry early resolve (parity, proof counts) and C3 on edited scenes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu exit $rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/r05_$tag.json \
    2> gpurun_out/r05_$tag.err
  local rc=$?; echo "bench $tag exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r05_$tag.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05_$tag.json')); r=d['roofline']; p=d['paths']; print('$tag', d['value'], r['kernel_ms'], r['frac'], p['rays_traced_per_sample'], p['shadow_proven_per_sample'])"
}
for i in 1 2; do
run c3_e$i
run c3_move_e$i --move-box 1
run c3_move_rt_e$i --move-box 1 --kernel-level cornell
done
