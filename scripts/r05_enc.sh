#!/usr/bin/env bash
# P3 encoder A/B (spt_image.hip p3_text staging): byte-exact image tests on the variant, then
# rocprofv3 kernel stats of tools/bench_image.py 4096 20 per build, 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SPT_LIB=build/ab/enc_plain.so timeout -k 10 300 python -u -m pytest tests/test_gpu_image.py tests/test_cpp_host.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/enc_tests.log 2>&1
rc=$?; echo "image tests (plain) exit $rc"; tail -2 gpurun_out/enc_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in base plain; do
    OUT=gpurun_out/enc_${v}_$r; mkdir -p $OUT
    SPT_LIB=build/ab/enc_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o enc -- python3 tools/bench_image.py 4096 20 > $OUT/log 2>&1 || { echo "$v rocprof failed"; exit 1; }
    python3 - "$OUT" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = {r["Name"].split("(")[0].split("::")[-1]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
print(sys.argv[2], {k: round(v, 1) for k, v in rows.items() if k.startswith(("p3", "p6", "pfm"))})
PY
  done
done | tee gpurun_out/enc_ab.txt
