set -e
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
timeout -k 10 120 python tools/ab_trace.py bunny,armadillo_proxy 100
AB_SHADOW=1 timeout -k 10 120 python tools/ab_trace.py merged_proxy,bunny 50
timeout -k 10 120 python tools/wave_timeline.py bunny | head -3
