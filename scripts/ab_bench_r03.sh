set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for b in bench_old_ab.py bench.py; do
  out=$(timeout -k 10 120 python $b --steps 10 --warmup 2 --no-cpu-baseline ${ARGS:-} 2>/dev/null) || { echo "$b FAILED"; exit 1; }
  echo "$b $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done; done
