# PMC passes over the bench's prefill (fused GEMM, flash attention): MFMA busy, then the wave-cycle breakdown
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_mfma -o pmc -- python3 tools/prefill_pmc.py > gpurun_out/pmc_mfma.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/pmc_waves -o pmc -- python3 tools/prefill_pmc.py > gpurun_out/pmc_waves.log 2>&1 || exit 1
python3 tools/prefill_pmc.py --summarize gpurun_out/pmc_mfma > gpurun_out/pmc_mfma_summary.txt 2>&1
python3 tools/prefill_pmc.py --dump gpurun_out/pmc_waves > gpurun_out/pmc_waves_summary.txt 2>&1
