# L2 behaviour of the prefill flash attention: hit / miss counts and the bytes the L2 fetched
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P="python3 tools/prefill_attn_bench.py"
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/fapmc4 -o pmc -- $P > gpurun_out/fapmc4.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/fapmc5 -o pmc -- $P > gpurun_out/fapmc5.log 2>&1 || exit 1
python3 tools/prefill_pmc.py --dump gpurun_out/fapmc4 > gpurun_out/fapmc_l2.txt 2>&1
python3 tools/prefill_pmc.py --dump gpurun_out/fapmc5 >> gpurun_out/fapmc_l2.txt 2>&1
