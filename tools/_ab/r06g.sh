bash tools/gpu_session.sh "r06g/e3_check:60:python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 2 --check"
