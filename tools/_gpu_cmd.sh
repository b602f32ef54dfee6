bash tools/gpu_build_diag.sh bdiag3
