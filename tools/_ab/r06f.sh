bash tools/gpu_session.sh \
 "r06f/e3_check:60:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 2 --check" \
 "r06f/ar_push:120:python -u tools/ar_push_time.py" \
 "r06f/e3_7b1:200:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 32 --floor" \
 "r06f/e3_7b8:200:python -u tools/lab/engine3/e3_ab.py --geom 7b8 --layers 32 --floor"
