"""CPU oracle for the lit_gpt quantized decode path — TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU, the reference algorithm of the hot path that the HIP kernels in
``lit-gpt_amd/csrc`` implement. It is the checker, never the thing
measured or shipped: only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it. The product path (``lit-gpt_amd/lit_gpt``) never imports it and
fails loudly when the HIP library is missing.

Pinning: ``tests/test_oracle_golden.py`` checks these functions against golden vectors produced by
running the reference itself (``/root/reference``, imported with stubs in this container) through
``tests/golden/make_golden.py``; the vectors are committed under ``tests/golden/``.

Modules:
  synth  — counter-based deterministic weights/prompts (no torch RNG; regenerable on any host)
  model  — fp32/bf16 restatement of GPT.forward, generate(), sample(), KV cache, RoPE, norms, MoE
  quant  — the build's int4-g128 and nf4-b64 weight formats: quantize / pack / dequantize (numpy)
  tp     — tensor_parallel_linear sharding restatement (generate/tp.py:28-45)
"""
