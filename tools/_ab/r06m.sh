bash tools/gpu_session.sh \
 "r06m/c3_check:90:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 2 --check" \
 @bench:r06m
