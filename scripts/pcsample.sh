#!/usr/bin/env bash
# rocprofv3 PC sampling of the render kernel (instruction hotspots). Output gpurun_out/pcs_<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
OUT=gpurun_out/pcs_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -i -B2 -A12 "pc_sampl\|PC Sampling" $OUT/avail.txt | head -60 > $OUT/pcs_caps.txt || true
for method in stochastic host_trap; do
  unit=cycles; [ $method = host_trap ] && unit=time
  interval=1048576; [ $method = host_trap ] && interval=100
  timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $method \
     --pc-sampling-unit $unit --pc-sampling-interval $interval --output-format csv \
     -d $OUT/$method -o pcs -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline \
     > $OUT/$method.log 2>&1
  rc=$?; echo "$method exit $rc"; tail -3 $OUT/$method.log
  if [ $rc -eq 0 ]; then break; fi
  if [ $rc -ne 1 ] && [ $rc -ne 2 ]; then exit $rc; fi
done
find $OUT -name "*.csv" | head
