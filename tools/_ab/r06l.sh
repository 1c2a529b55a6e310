bash tools/gpu_session.sh \
 "r06l/c3_check:90:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 2 --check" \
 "r06l/c3_7b1:240:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 32 --trace"
