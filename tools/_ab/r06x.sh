bash tools/gpu_session.sh \
 "r06x/7b_variants:300:GEMV_VARIANTS=-1,0,8,1,-1,8 python -u tools/gemv_variants.py lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so"
