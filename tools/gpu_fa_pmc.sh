# PMC passes over the prefill flash-attention timing program: MFMA busy, wave-cycle breakdown, LDS
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P="python3 tools/prefill_attn_bench.py"
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/fapmc1 -o pmc -- $P > gpurun_out/fapmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/fapmc2 -o pmc -- $P > gpurun_out/fapmc2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/fapmc3 -o pmc -- $P > gpurun_out/fapmc3.log 2>&1 || exit 1
python3 tools/prefill_pmc.py --summarize gpurun_out/fapmc1 > gpurun_out/fapmc_summary.txt 2>&1
python3 tools/prefill_pmc.py --dump gpurun_out/fapmc2 >> gpurun_out/fapmc_summary.txt 2>&1
python3 tools/prefill_pmc.py --dump gpurun_out/fapmc3 >> gpurun_out/fapmc_summary.txt 2>&1
