bash tools/gpu_session.sh \
 "r06q/same_r4:120:AB_LIBS=tools/_ab/liblitgpt_r4c7.so,tools/_ab/liblitgpt_r4c7b.so python -u tools/moe_down_ab.py" \
 "r06q/same_c8:120:AB_LIBS=tools/_ab/liblitgpt_cpt8.so,tools/_ab/liblitgpt_cpt8b.so python -u tools/moe_down_ab.py" \
 "r06q/r2_first:120:AB_LIBS=tools/_ab/liblitgpt_r2c7.so,tools/_ab/liblitgpt_r4c7.so,tools/_ab/liblitgpt_cpt8.so python -u tools/moe_down_ab.py"
