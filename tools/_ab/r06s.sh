bash tools/gpu_session.sh \
 "r06s/gemv_ab:300:python -u tools/gemv_variants.py tools/_ab/liblitgpt_pre_sched.so lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so tools/_ab/liblitgpt_pre_sched.so lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so" \
 "r06s/tests:400:python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -q -x -k 'gemv or stream or argmax or lm_head or greedy or decode' --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "r06s/bench:300:python -u bench.py --no-cpu-baseline --no-traffic"
