bash tools/gpu_session.sh \
 "r06w/fc_variants:240:python -u tools/moe_fc_variants.py -1,0,1,8,17,33,49"
