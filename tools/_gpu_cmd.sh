set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD; OUT=$ROOT/gpurun_out/nrm2; mkdir -p $OUT
for i in 1 2 3; do
timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy >> $OUT/n128.log 2>&1 || exit 3
BEAM_HIP_LIB=$ROOT/raytracercuda_amd/libbeam_hip_n256.so timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy >> $OUT/n256.log 2>&1 || exit 4
BEAM_HIP_LIB=$ROOT/raytracercuda_amd/libbeam_hip_n448.so timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy >> $OUT/n448.log 2>&1 || exit 5
BM_NRM_DEFER=0 timeout -k 10 120 python tools/build_bench.py bunny,armadillo_proxy,merged_proxy >> $OUT/old.log 2>&1 || exit 6
done
echo ok
