bash tools/gpu_session.sh \
 "r06zb/tests:600:python -u -m pytest tests -m gpu -q -x -k 'gemv or moe or pair or expert or Mixtral or gate or route or tp' --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "r06zb/bench_mix:300:python -u bench.py --model Mixtral-8x7B-v0.1 --no-cpu-baseline --no-traffic"
