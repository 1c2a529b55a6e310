AB="AB_LIBS=lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so,tools/_ab/liblga_attn_nofix.so"
bash tools/gpu_session.sh \
 "r06b/attn_ab_7b:300:$AB AB_POS=2063,2183,2302 python -u tools/attn_ab.py" \
 "r06b/attn_ab_mix:300:$AB AB_HEADS=32 AB_GROUPS=8 AB_POS=2063,2302 python -u tools/attn_ab.py" \
 "r06b/attn_ab_tp8:300:$AB AB_HEADS=4 AB_GROUPS=4 AB_POS=2063,2302 python -u tools/attn_ab.py" \
 "r06b/e3_check:120:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 4 --check" \
 "r06b/e3_7b1:200:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 32 --floor" \
 "r06b/e3_7b8:200:python -u tools/lab/engine3/e3_ab.py --geom 7b8 --layers 32 --floor" \
 "r06b/ar_push:200:GPU_MAX_HW_QUEUES=4 python -u tools/ar_push_time.py"
