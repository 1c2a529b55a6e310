#!/bin/bash
# round-3 second session: new-feature GPU tests, decode-attention A/B (old contiguous chunks / row-run prefetch /
# + tagged publish), then the default bench line
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
exec bash tools/gpu_session.sh \
  "t_kernels:600:$T tests/test_gpu_kernels.py tests/test_gpu_gemm_fused.py" \
  "t_neox:400:$T tests/test_gpu_neox.py" \
  "t_tp:700:$T tests/test_gpu_tp.py -k 'fused_gemv or bit_exact or tp2'" \
  "attn_ab:300:ATTN_LIBS=tools/_lab/attn_old.so,tools/_lab/attn_new.so,tools/_lab/attn_tag.so ATTN_MODE=fused ATTN_SPLITS=8 python -u tools/attn_sweep.py" \
  "bench:400:python -u bench.py --no-cpu-baseline"
