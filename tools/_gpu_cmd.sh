set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r05_v5; mkdir -p $OUT
for r in 1 2; do
 for v in libbeam_hip.so libbeam_hip_htop.so libbeam_hip_sa.so; do
  echo "-- $v $r"; BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$v timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy 2>&1 | grep -v amdgpu.ids || exit 4
 done
done
for v in libbeam_hip_bdiag.so libbeam_hip_sa_bdiag.so; do
  echo "== diag $v"; BEAM_HIP_LIB=$(pwd)/raytracercuda_amd/$v timeout -k 10 120 python tools/build_diag.py bunny,armadillo_proxy,merged_proxy 2>&1 | grep -v amdgpu.ids || exit 5
done
