bash tools/gpu_session.sh \
 "r06k/c3_check:90:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 2 --check" \
 "r06k/c3_7b1:240:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 32 --trace --floor" \
 "r06k/c9_7b1:240:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 32 --trace --lib liblga_engine3_c9.so --esplits 3" \
 "r06k/c6_7b1:240:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 32 --lib liblga_engine3_c6.so --esplits 3"
