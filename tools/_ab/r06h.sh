bash tools/gpu_session.sh \
 "r06h/e3_check:60:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 2 --check" \
 "r06h/e3_7b1:200:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 32 --floor" \
 "r06h/e3_7b8:200:python -u tools/lab/engine3/e3_ab.py --geom 7b8 --layers 32 --floor"
