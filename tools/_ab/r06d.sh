bash tools/gpu_session.sh \
 "r06d/e3_check:60:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 2 --check" \
 "r06d/ar_push:120:python -u tools/ar_push_time.py" \
 "r06d/ar_push_informal:120:LGA_LIB=tools/_ab/liblga_ar_informal.so python -u tools/ar_push_time.py" \
 "r06d/tp_fused_tests:500:python -u -m pytest tests/test_gpu_tp.py -x -v --timeout 300 -k fused_gemv_allreduce -p no:cacheprovider" \
 "r06d/e3_7b1:200:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 32 --floor"
