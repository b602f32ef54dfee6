#!/usr/bin/env bash
# One-GPU rehearsal of the N>1 bench path (all ranks on cuda:0, gloo carries the bands):
#   tools/gpu_rehearse.sh TAG  -> gpurun_out/TAG/n2_c2.log, n4_c4.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="gpurun_out/${1:-rehearse}"; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 BM_BENCH_SHARED_DEVICE=1
for nc in "2 c2 29611" "4 c4 29612" "3 c5 29613"; do
  set -- $nc
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 \
    --master-port $3 bench.py --gpus $1 --config $2 --steps 10 --warmup 3 > "$OUT/n$1_$2.log" 2>&1
  rc=$?; echo "== n$1 $2 rc=$rc"; grep '^{' "$OUT/n$1_$2.log" | cut -c1-200
  if [ $rc -ne 0 ]; then tail -5 "$OUT/n$1_$2.log"; exit $rc; fi
done
