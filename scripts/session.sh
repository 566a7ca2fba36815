#!/usr/bin/env bash
# Measurement session on the GPU box (in-tree build): GPU tests, the C3 rocprofv3 session (kernel
# trace + separate PMC passes, scripts/profile.sh), instruction-class PMC passes, and the bench lines
# of every config (C2-C5, with their CPU baselines). Outputs are tagged with TAG (default r04).
#   PARTS="record pytest smoke rehearsal profile classes waves dropin levels bench" selects parts;
#   each GPU step has its own time limit and the script stops at the first failure.
#   record: scripts/gpu_record.py TAG (pytest -m gpu + smoke, stamped; SPT_GIT_HEAD from the caller)
#   waves:  per-wave dumps of C2 and C3 with the SPT_DIAG=2 build (build/ab/diag2.so, made by
#           scripts/build_variants.sh diag2:"-DSPT_DIAG=2" beforehand) -> gpurun_out/TAG_waves_*.json
#   levels: scripts/levels.sh (kernel levels at C3 / C2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PARTS=${PARTS:-"pytest profile classes bench"}
TAG=${TAG:-r04}
has() { case " $PARTS " in *" $1 "*) return 0;; esac; return 1; }
if has record; then
  timeout -k 10 900 python -u scripts/gpu_record.py $TAG > gpurun_out/${TAG}_record.log 2>&1
  rc=$?; echo "gpu_record exit $rc"; tail -2 gpurun_out/${TAG}_record.log; [ $rc -eq 0 ] || exit $rc
fi
if has pytest; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest -m gpu exit $rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke exit $rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if has rehearsal; then  # the N>1 bench path on the one GPU (gloo gather; RCCL needs one GPU per rank)
  RANKS="${RANKS:-2 4}" bash scripts/rehearsal.sh || exit $?
fi
if has profile; then
  bash scripts/profile.sh $TAG || exit $?
fi
if has classes; then
  # CLS: configurations (tag[:chunk]); c2:32 = C2 at 32-sample units (the C2 tail study)
  for spec in ${CLS:-c3 c5}; do
    cfg=${spec%%:*}; tag=$cfg
    args="--steps 2 --warmup 1 --no-cpu-baseline --no-extras --config $cfg"
    [ $cfg = c5 ] && args="$args --spp 256"
    case $spec in *:*) args="$args --chunk ${spec#*:}"; tag=${cfg}_u${spec#*:};; esac
    mkdir -p gpurun_out/cls_$tag; cfg=$tag
    i=0
    for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM" \
               "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE" \
               "SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_IFETCH SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FLOPS_FP32" \
               "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT" ; do
      i=$((i+1)); [ $i -le ${CLS_PASSES:-4} ] || break
      timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/cls_$cfg/p$i -o p$i \
        -- python3 bench.py $args > gpurun_out/cls_$cfg/p$i.log 2>&1; rc=$?
      echo "$cfg class pass $i exit $rc"; [ $rc -eq 0 ] || exit $rc
    done
    python3 scripts/pmc_summary.py gpurun_out/cls_$cfg > gpurun_out/cls_$cfg/summary.json
  done
fi
if has waves; then
  for cfg in c2 c3; do
    SPT_LIB=build/ab/diag2.so timeout -k 10 180 python tools/wave_dump.py $cfg gpurun_out/${TAG}_waves_$cfg.bin \
      > gpurun_out/${TAG}_waves_$cfg.json 2> gpurun_out/${TAG}_waves_$cfg.err
    rc=$?; echo "waves $cfg exit $rc"; [ $rc -eq 0 ] || exit $rc
  done
fi
if has levels; then
  TAG=$TAG bash scripts/levels.sh || exit $?
fi
if has dropin; then  # the drop-in program end to end (tools/dropin_e2e.py) and its kernels under rocprofv3
  timeout -k 10 600 python tools/dropin_e2e.py --ref-spp 8 --out gpurun_out/${TAG}_dropin.json \
    > gpurun_out/dropin.log 2>&1
  rc=$?; echo "dropin exit $rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/dropin.log; exit $rc; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dropin -o dropin \
    -- small-pathtracer_amd/smallpt_amd 1024 768 512 1 /tmp/dropin.ppm --repeat 10 > gpurun_out/prof_dropin.log 2>&1
  rc=$?; echo "dropin rocprof exit $rc"; [ $rc -eq 0 ] || exit $rc
fi
if has bench; then
  for cfg in c3 c2 c4 c5; do
    st=5; [ $cfg = c4 ] && st=3; [ $cfg = c5 ] && st=2
    timeout -k 10 420 python bench.py --config $cfg --steps $st --warmup 1 \
      > gpurun_out/${TAG}_bench_$cfg.json 2> gpurun_out/${TAG}_bench_$cfg.err
    rc=$?; echo "bench $cfg exit $rc"; [ $rc -eq 0 ] || exit $rc
  done
fi
