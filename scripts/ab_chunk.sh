#!/usr/bin/env bash
# Unit size vs time and memory-side atomic traffic on C3: bench timing per --chunk, then one
# rocprofv3 --pmc WRITE_SIZE pass each. Usage: scripts/ab_chunk.sh CHUNK... (0 = auto)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_chunk
export TMPDIR=/tmp
for r in 1 2; do
  for c in "$@"; do
    out=$(timeout -k 10 120 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --chunk $c 2>/dev/null) || { echo "chunk $c FAILED"; exit 1; }
    echo "chunk $c $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done | tee gpurun_out/ab_chunk/times.txt
for c in "$@"; do
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/ab_chunk/w$c -o w$c -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --chunk $c > gpurun_out/ab_chunk/w$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
  python3 - "$c" <<'PY'
import csv, glob, sys
c = sys.argv[1]
f = glob.glob(f"gpurun_out/ab_chunk/w{c}/**/*counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "render_kernel" in r["Kernel_Name"]]
print(f"chunk {c} WRITE_SIZE per render launch (KB, mean of {len(v)}): {sum(v)/len(v):.0f}")
PY
done | tee gpurun_out/ab_chunk/traffic.txt
