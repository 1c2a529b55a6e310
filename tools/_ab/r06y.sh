mkdir -p gpurun_out/r06y && bash tools/gpu_session.sh \
 "r06y/e3_dump:120:E3_ATTN_DUMP=gpurun_out/r06y/e3_attn.npz python -u tools/lab/engine3/e3_ab.py --geom 7b1 --layers 2 --check"
