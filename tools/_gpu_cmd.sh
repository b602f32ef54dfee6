set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v22; mkdir -p $OUT
timeout -k 10 120 python tools/host_rate.py c3 c2 c5 2>&1 | grep -v "amdgpu.ids" || exit 4
