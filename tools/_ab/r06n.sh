bash tools/gpu_session.sh \
 "r06n/save_w8:120:python -u tools/q4f_tile_ab.py save /tmp/w8.pt" \
 "r06n/save_w4:120:LGA_Q4F_W4=1 python -u tools/q4f_tile_ab.py save /tmp/w4.pt" \
 "r06n/compare:60:python -u tools/q4f_tile_ab.py compare /tmp/w8.pt /tmp/w4.pt" \
 "r06n/rates_w8:180:python -u tools/gemm_rates.py 2048" \
 "r06n/rates_w4:180:LGA_Q4F_W4=1 python -u tools/gemm_rates.py 2048" \
 "r06n/tests_w4:400:LGA_Q4F_W4=1 python -u -m pytest tests/test_gpu_gemm_fused.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "r06n/bench_w4:300:LGA_Q4F_W4=1 python -u bench.py --no-cpu-baseline --no-traffic" \
 "r06n/bench_w8:300:python -u bench.py --no-cpu-baseline --no-traffic"
