bash tools/gpu_session.sh \
 "r06j/c9_check:90:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 2 --check --lib liblga_engine3_c9.so --esplits 3" \
 "r06j/c9_7b1:240:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 32 --trace --lib liblga_engine3_c9.so --esplits 3" \
 "r06j/c6_7b1:240:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 32 --lib liblga_engine3_c6.so --esplits 3" \
 "r06j/c9_7b8:240:python -u tools/lab/engine3/e3_ab.py --geom 7b8 --layers 32 --lib liblga_engine3_c9.so"
