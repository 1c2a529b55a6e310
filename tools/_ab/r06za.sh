bash tools/gpu_session.sh \
 "r06za/down_nw8:180:AB_LIBS=lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so,tools/_ab/liblitgpt_pair_nw8.so python -u tools/moe_down_ab.py"
