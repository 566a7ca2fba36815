#!/usr/bin/env bash
# Round-3 P3 encoder session: byte-exact image tests, then rocprofv3 kernel trace of the encoder
# microbench (tools/bench_image.py, 4096^2) for the in-tree build and the A/B builds in LIBS
# (e.g. build/ab/p3single.so from scripts/build_variants.sh p3single:"-DSPT_P3_SINGLE=1").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_image.py tests/test_cpp_host.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/enc_tests.log 2>&1
rc=$?; echo "image tests exit $rc"; tail -3 gpurun_out/enc_tests.log; [ $rc -eq 0 ] || exit $rc
libs="small-pathtracer_amd/libspt.so ${LIBS:-}"
for lib in $libs; do
  name=$(basename $lib .so)
  SPT_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/enc_$name -o enc \
    -- python3 tools/bench_image.py 4096 10 > gpurun_out/enc_$name.log 2>&1
  rc=$?; echo "$name rocprof exit $rc"; [ $rc -eq 0 ] || exit $rc
  grep p3 gpurun_out/enc_$name.log
done
