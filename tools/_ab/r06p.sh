bash tools/gpu_session.sh \
 "r06p/down_ab:180:AB_LIBS=lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so,tools/_lab/liblitgpt_cpt8.so python -u tools/moe_down_ab.py" \
 "r06p/moe_tests:400:python -u -m pytest tests -m gpu -q -x -k 'moe or pair or mixtral or Mixtral or expert' --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "r06p/mixtral_bench:400:python -u bench.py --model Mixtral-8x7B-v0.1 --no-traffic --no-cpu-baseline"
