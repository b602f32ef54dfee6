set -e
export BM_BENCH_SHARED_DEVICE=1
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --steps 10 --warmup 3 > gpurun_out/rehearsal_$n.log 2>&1 || { tail -30 gpurun_out/rehearsal_$n.log; exit 1; }
  grep '^{' gpurun_out/rehearsal_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['value'], d['n_gpus'], d.get('frame_check'), d.get('frame_hits'), d['config']['workload'])"
done
