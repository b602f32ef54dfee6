#!/usr/bin/env bash
# The driver's N>1 bench commands rehearsed on a one-GPU box: N ranks share cuda:0 and gather over
# gloo (BM_BENCH_SHARED_DEVICE=1; RCCL refuses two ranks on one device). Each line must report the
# fixed frame (1920x1080 for c2, 3840x2160 for c4) with frame_check true on every gathered plane.
#   tools/gpu_scale_rehearsal.sh [N list, default "2 4"] [configs, default "c2 c4"]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 BM_BENCH_SHARED_DEVICE=1
OUT=gpurun_out/scale; mkdir -p $OUT
for cfg in ${2:-c2 c4}; do for N in ${1:-2 4}; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus $N --steps 6 --warmup 2 --config $cfg > $OUT/${cfg}_n$N.log 2>&1 || exit $?
  tail -1 $OUT/${cfg}_n$N.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$cfg', d['n_gpus'], c['width'], c['height'], d['frame_check'], d['checked_planes'], d['scaling'], c['workload'][:150])"
done; done
