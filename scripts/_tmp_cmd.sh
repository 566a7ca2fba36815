set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 90 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke0.log 2>&1 || { echo "smoke failed $?"; tail -5 gpurun_out/smoke0.log; exit 3; }
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=2 bash scripts/ab.sh build/ab/f0.so build/ab/v4.so
