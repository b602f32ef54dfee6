set -u
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
PMC_GROUPS=tools/pmc_groups3.txt bash tools/pmc_trace.sh ${1:-pmc_core} ${2:-bunny}
python3 tools/pmc_summary.py gpurun_out/${1:-pmc_core} > gpurun_out/${1:-pmc_core}/summary.txt 2>&1 || true
