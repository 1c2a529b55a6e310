# cold-prefill diagnosis: wall times in both orders, then a kernel + HIP API trace of the bench's order
set -o pipefail
mkdir -p gpurun_out/cold
timeout -k 10 300 python -u tools/prefill_cold.py --order big-first > gpurun_out/cold/big.log 2>&1 && \
timeout -k 10 300 python -u tools/prefill_cold.py --order small-first > gpurun_out/cold/small.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --output-format csv -d gpurun_out/cold/prof -o cold -- python tools/prefill_cold.py --order big-first > gpurun_out/cold/prof.log 2>&1
