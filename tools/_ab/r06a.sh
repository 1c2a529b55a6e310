AB="AB_LIBS=lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so,tools/_ab/liblga_attn_nofix.so"
bash tools/gpu_session.sh @tests:r06a @bench:r06a \
 "r06a/attn_ab_7b:300:$AB AB_POS=2063,2183,2302 python -u tools/attn_ab.py" \
 "r06a/attn_ab_mix:300:$AB AB_HEADS=32 AB_GROUPS=8 AB_POS=2063,2302 python -u tools/attn_ab.py" \
 "r06a/attn_ab_tp8:300:$AB AB_HEADS=4 AB_GROUPS=4 AB_POS=2063,2302 python -u tools/attn_ab.py"
