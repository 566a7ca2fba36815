#!/usr/bin/env bash
# The driver's round-end forms with the final build: smoke(), then bench.py with no arguments.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -1 gpurun_out/smoke_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_default.err; exit $rc; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench_default.json"))
r = d["roofline"]
print(d["config"]["workload"], d["value"], d["steps"], d["warmup"], r["kernel_ms"], r["frac"], r.get("frac_hw"),
      d["cpu_baseline"]["value"])
PY
