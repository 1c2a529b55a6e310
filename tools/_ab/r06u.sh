bash tools/gpu_session.sh \
 "r06u/tests:500:python -u -m pytest tests -m gpu -q -x -k 'gemv or moe or pair or expert or Mixtral or gate or route or tp' --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "r06u/mix_variants:200:GEMV_SHAPES=mixtral python -u tools/gemv_variants.py tools/_ab/liblitgpt_pre_half.so lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so" \
 "r06u/bench_mix:300:python -u bench.py --model Mixtral-8x7B-v0.1 --no-cpu-baseline --no-traffic" \
 "r06u/bench:300:python -u bench.py --no-cpu-baseline --no-traffic"
