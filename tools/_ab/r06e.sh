bash tools/gpu_session.sh \
 "r06e/e3_check:60:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 2 --check" \
 "r06e/tp_fused_tests:400:python -u -m pytest tests/test_gpu_tp.py -x -v --timeout 120 -k 'fused_gemv_allreduce and tagged' -p no:cacheprovider"
