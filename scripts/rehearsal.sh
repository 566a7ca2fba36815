#!/usr/bin/env bash
# 4- and 8-rank (RANKS="2 4 8" for more) rehearsals of the multi-GPU bench on the one GPU (gloo gather through host memory;
# RCCL refuses two ranks on one device): every rank renders its cyclic 8-row tiles of the C3
# image at N x 512 spp, rank 0 gathers, re-renders the whole image alone and compares bit for bit.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for n in ${RANKS:-4 8}; do
  timeout -k 10 300 env SPT_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 2 --warmup 1 \
    --no-cpu-baseline --verify-gather > gpurun_out/rehearsal$n.log 2>&1 || exit $?
  grep '^{' gpurun_out/rehearsal$n.log | tail -1 > gpurun_out/rehearsal$n.json
  python3 -c "import json; d=json.load(open('gpurun_out/rehearsal$n.json')); print($n, d['value'], d['config']['spp'], d['gather_equals_1gpu_render'])"
done
