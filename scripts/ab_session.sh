set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/classic_anchor.py --spp 1024 --png gpurun_out/classic.png > gpurun_out/classic_anchor.json 2>gpurun_out/classic_anchor.err || exit $?
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -k "classic" --timeout 100 --timeout-method thread > gpurun_out/classic_tests.log 2>&1 || exit $?
tail -3 gpurun_out/classic_tests.log
