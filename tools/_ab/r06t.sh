bash tools/gpu_session.sh \
 "r06t/mix_variants:300:GEMV_SHAPES=mixtral GEMV_VARIANTS=-1,0,8,1,-1,8 python -u tools/gemv_variants.py lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so"
