bash tools/gpu_session.sh \
 "r06o/mixtral_prof:400:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06o/prof -o mix -- python bench.py --model Mixtral-8x7B-v0.1 --no-traffic --no-cpu-baseline --no-sample"
