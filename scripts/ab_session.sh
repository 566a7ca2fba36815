set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
BENCH_ARGS="--config c5 --spp 256" ROUNDS=2 timeout -k 10 400 bash scripts/ab.sh build/ab/g64.so build/ab/u8.so build/ab/u6.so build/ab/u4.so > gpurun_out/ab_c5.txt 2>&1 || exit $?
BENCH_ARGS="--config c3" ROUNDS=2 timeout -k 10 300 bash scripts/ab.sh build/ab/g64.so build/ab/u8.so > gpurun_out/ab_c3.txt 2>&1 || exit $?
cat gpurun_out/ab_c5.txt gpurun_out/ab_c3.txt
