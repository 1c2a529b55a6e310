#!/bin/bash
# MFMA-busy PMC pass over the bench's prefill (final tree)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_mfma -o pmc -- python3 tools/prefill_pmc.py > gpurun_out/pmc_mfma.log 2>&1 || exit 1
python3 tools/prefill_pmc.py --summarize gpurun_out/pmc_mfma > gpurun_out/pmc_mfma_summary.txt 2>&1
