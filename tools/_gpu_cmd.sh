set -e
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/pt.log 2>&1 || { tail -40 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
