#!/usr/bin/env bash
# Rehearsal of bench.py's N-rank path on a one-GPU box: N ranks share cuda:0, gloo instead of RCCL
# (BM_BENCH_SHARED_DEVICE=1, the gather stages through host memory). Checks frame_check only; the
# timing means nothing. Usage: bash tools/gpu_multi_rehearsal.sh [N=2] [planes=packed]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 BM_BENCH_SHARED_DEVICE=1
N=${1:-2}; P=${2:-packed}
mkdir -p gpurun_out/multi
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus $N --steps 10 --warmup 3 --gather-planes $P > gpurun_out/multi/n$N.log 2>&1
rc=$?; grep -o '"frame_check": [a-z]*\|"n_gpus": [0-9]*\|"value": [0-9.]*' gpurun_out/multi/n$N.log; tail -3 gpurun_out/multi/n$N.log | cut -c1-300; exit $rc
