bash tools/gpu_session.sh \
 "r06c/e3_check:60:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 2 --check" \
 "r06c/ar_push_informal:120:LGA_LIB=tools/_ab/liblga_ar_informal.so python -u tools/ar_push_time.py"
