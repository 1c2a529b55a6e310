bash tools/gpu_session.sh \
 "r06r/gemv_ab:300:python -u tools/gemv_variants.py tools/_ab/liblitgpt_pre_bfly.so lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so tools/_ab/liblitgpt_pre_bfly.so lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so" \
 "r06r/down_ab:180:AB_LIBS=lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so,tools/_ab/liblitgpt_cpt8.so,tools/_ab/liblitgpt_pre_bfly.so python -u tools/moe_down_ab.py" \
 "r06r/tests:600:python -u -m pytest tests -m gpu -q -x -k 'gemv or moe or pair or expert or Mixtral or tp' --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "r06r/bench:300:python -u bench.py --no-cpu-baseline --no-traffic" \
 "r06r/bench_mix:300:python -u bench.py --model Mixtral-8x7B-v0.1 --no-cpu-baseline --no-traffic"
