set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for c in c2 c3; do
BENCH_ARGS="--config $c" ROUNDS=2 timeout -k 10 300 bash scripts/ab.sh build/ab/g64.so build/ab/guided.so build/ab/base.so > gpurun_out/ab_$c.txt 2>&1 || exit $?
done
BENCH_ARGS="--config c4" ROUNDS=1 timeout -k 10 300 bash scripts/ab.sh build/ab/g64.so build/ab/guided.so build/ab/base.so > gpurun_out/ab_c4.txt 2>&1 || exit $?
BENCH_ARGS="--config c5 --spp 256" ROUNDS=1 timeout -k 10 300 bash scripts/ab.sh build/ab/g64.so build/ab/guided.so build/ab/base.so > gpurun_out/ab_c5.txt 2>&1 || exit $?
for c in c2 c3 c4 c5; do echo "== $c"; cat gpurun_out/ab_$c.txt; done
