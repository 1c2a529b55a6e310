"""Decode benchmark: Llama-2-7B int4-g128, single-stream greedy decode at context 2048 (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
N > 1 is launched by the driver as ``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...``
and runs tensor parallelism (generate/tp.py sharding, RCCL all-reduce): one stream, so ``value`` is that stream's
tokens/s (whole job) and scaling is "strong".

A "step" = one decode token: one replay of the captured HIP graph (32 blocks + lm_head + argmax) at positions
2048 + W ... 2048 + W + K - 1 after a 2048-token synthetic prefill. Inputs (weights, KV cache, token, position)
are resident in HBM before the timed region. Timed region: barrier + synchronize, K replays, synchronize +
barrier; the max over ranks is reported.

Extra objects in the JSON line:
  roofline      the dominant kernel = the one with the most device time per decode step, chosen in the run
                between the decode attention (RoPE + KV append + split attention, K/V bytes at the timed
                position) and the fused RMSNorm + fc_1/fc_2 int4 GEMV + SwiGLU (46.5 MB per launch); each is
                timed with HIP events on the launch stream (all 32 blocks back to back in a HIP graph); peak
                8 TB/s; traffic = HBM bytes per launch from a rocprofv3 FETCH_SIZE pass at the same position.
                roofline_secondary = the other one
  step_roofline the whole decode step: algorithmic bytes per token (weights + KV read/write) x tok/s
  cpu_baseline  the CPU oracle (restatement of the reference's bf16 math) timed on this host on a bounded sample
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent
for _p in (str(REPO / "lit-gpt_amd"), str(REPO)):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
MODEL = "Llama-2-7b-hf"
PROMPT_LEN = 2048
CHUNK = 8  # decode steps per graph launch (generate/base.py DECODE_CHUNK)


def algorithmic_bytes_per_token(cfg, pos: float, group: int = 128, tp: int = 1, dense: bool = False) -> float:
    """Weights (all Linears incl. lm_head, int4 + bf16 group scale, or bf16 when ``dense``) + norms + embedding
    row + KV read/write, per rank (SURVEY §8d formula). Sparse MoE blocks count the router and the k routed
    experts only."""
    C, V, L = cfg.n_embd, cfg.padded_vocab_size, cfg.n_layer
    qkv = (cfg.n_head + 2 * cfg.n_query_groups) * cfg.head_size
    mlp = 3 * cfg.intermediate_size * C
    per_layer = (qkv * C + C * C) / tp
    if cfg._mlp_class == "LLaMAMoE":
        per_layer += cfg.n_expert * C + cfg.n_expert_per_token * mlp / tp  # gate replicated, experts sliced
    else:
        per_layer += mlp / tp
    bw = 2.0 if dense else 0.5 + 2.0 / group
    weights = (L * per_layer + V * C) * bw
    norms = (2 * L + 1) * C * 2
    kv = 2 * L * (cfg.n_query_groups / tp) * cfg.head_size * 2 * (pos + 1) + 2 * L * (cfg.n_query_groups / tp) * cfg.head_size * 2
    return weights + norms + C * 2 + kv


MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)


def prefill_flops(cfg, T: int, tp: int = 1) -> float:
    """Algorithmic FLOPs of one T-token prefill with last_token_only: 2*T*sum(N*K) over the blocks'
    Linears (MoE: the k routed experts per token + the router), causal attention 2*2*H*hs*T*(T+1)/2 per layer
    (QK^T and P.V over the keys each query sees), and the lm_head for the last row only; per rank."""
    C, L = cfg.n_embd, cfg.n_layer
    qkv = (cfg.n_head + 2 * cfg.n_query_groups) * cfg.head_size
    mlp = 3 * cfg.intermediate_size * C
    per_tok = (qkv * C + C * C) / tp
    if cfg._mlp_class == "LLaMAMoE":
        per_tok += cfg.n_expert * C + cfg.n_expert_per_token * mlp / tp
    else:
        per_tok += mlp / tp
    attn = 2.0 * 2.0 * (cfg.n_head / tp) * cfg.head_size * T * (T + 1) / 2
    return L * (2.0 * T * per_tok + attn) + 2.0 * cfg.padded_vocab_size * C


DOMINANT = "gemv_q4s_kernel<.., DUAL> (streaming form: RMSNorm + fc_1/fc_2 int4 GEMV + SwiGLU of one block)"


def time_attention(model, pos: int, replays: int = 5):
    """Average launch duration of the decode attention (RoPE + KV append + split attention, one launch per block)
    over the blocks' own KV caches at position ``pos`` — the second-largest per-step kernel — with HIP events on
    the launch stream (32 launches captured back to back in a HIP graph). Returns (ms, algorithmic bytes per
    launch): K and V rows 0..pos of every query group + the qkv row in + the attention row out."""
    from lit_gpt import ops

    blocks = model.transformer.h
    c = blocks[0].attn.config  # this rank's heads under tensor parallelism
    H, G, hs = c.n_head, c.n_query_groups, c.head_size
    if not ops.decode_fusable(hs, c.rope_n_elem) or blocks[0].attn.kv_cache is None:
        return None, None
    cos, sin = model._rope_tables()
    qkv = torch.randn(1, (H + 2 * G) * hs, device="cuda").to(torch.bfloat16)
    p = torch.tensor([pos], device="cuda")
    S = blocks[0].attn.kv_cache.k.size(-2)
    splits = ops.decode_splits(G, H // G, hs, S)
    ws = ops.AttentionWorkspace(1, H, G, hs, splits, torch.device("cuda", torch.cuda.current_device()))
    out = torch.empty(1, H * hs, device="cuda", dtype=torch.bfloat16)

    def launch_all():
        for blk in blocks:
            kv = blk.attn.kv_cache
            ops.attention_decode_fused(qkv, kv.k, kv.v, p, p, cos, sin, H, G, hs, c.rope_n_elem, 1.0 / math.sqrt(hs),
                                       splits, workspace=ws, out=out)

    launch_all()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        launch_all()
    graph.replay()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    for _ in range(replays):
        graph.replay()
    e.record(stream)
    e.synchronize()
    nbytes = 2 * G * hs * 2 * (pos + 1) + (H + 2 * G) * hs * 2 + H * hs * 2
    return s.elapsed_time(e) / (replays * len(blocks)), nbytes


def _dual_gemv_bytes(f1, C: int) -> int:
    """Algorithmic bytes of one dual-GEMV launch: both packed weight matrices + their group scales, the norm weight,
    x, and the bf16 output (kernel table)."""
    return (2 * f1.qweight.numel() + 2 * f1.scales.numel() * f1.scales.element_size() + 2 * C * 2
            + f1.out_features * 2)


def time_dominant_kernel(model, replays: int = 5):
    """Average launch duration of the dominant kernel, measured with HIP events on the stream the launches run on:
    the fused RMSNorm + fc_1/fc_2 + SwiGLU GEMV of every block (32 distinct 46.5 MB weight sets, 1.5 GB, so every
    launch streams from HBM as in the decode step), captured back to back in one HIP graph and replayed. Sparse
    MoE blocks: the routed form (two experts, ids 0 and 1) of the same kernel."""
    from lit_gpt import ops
    from lit_gpt.model import LLaMAMoE

    blocks = model.transformer.h
    moe = isinstance(blocks[0].mlp, LLaMAMoE)
    f1 = blocks[0].mlp.experts[0].fc_1 if moe else blocks[0].mlp.fc_1
    C = f1.in_features
    dense = type(f1) is torch.nn.Linear
    x = torch.randn(C, device="cuda").to(torch.bfloat16)
    ids = torch.tensor([0, 1], dtype=torch.int32, device="cuda")
    out = torch.empty(2 if moe else 1, f1.out_features, dtype=torch.bfloat16, device="cuda")

    def launch_all():
        for blk in blocks:
            if moe:
                (q1, s1), (q2, s2), _ = blk.mlp._stack()
                ops.q4_gemv_swiglu_experts(x, q1, s1, q2, s2, ids, f1.out_features, C, f1.group, f1.fmt,
                                           norm_weight=blk.norm_2.weight, eps=blk.norm_2.eps, out=out)
                continue
            a, b = blk.mlp.fc_1, blk.mlp.fc_2
            if dense:
                ops.bf16_gemv_swiglu(x, a.weight, b.weight, norm_weight=blk.norm_2.weight, eps=blk.norm_2.eps,
                                     out=out.view(-1))
                continue
            ops.q4_gemv_swiglu(x, a.qweight, a.scales, b.qweight, b.scales, a.out_features, C, a.group, a.fmt,
                               norm_weight=blk.norm_2.weight, eps=blk.norm_2.eps, out=out.view(-1))

    launch_all()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        launch_all()
    graph.replay()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    for _ in range(replays):
        graph.replay()
    e.record(stream)
    e.synchronize()
    avg_ms = s.elapsed_time(e) / (replays * len(blocks))
    if dense:
        return avg_ms, 2 * f1.weight.numel() * 2 + 2 * C * 2 + f1.out_features * 2
    return avg_ms, _dual_gemv_bytes(f1, C) * (2 if moe else 1)


def pmc_child(att_pos: int) -> None:
    """Run under `rocprofv3 --pmc FETCH_SIZE` by measure_traffic(): the fc_1||fc_2 GEMV at Llama-2-7B shape over
    24 distinct weight sets (1.1 GB, beyond the 256 MB Infinity Cache), one launch each, then the decode attention
    over 24 distinct K/V caches at position ``att_pos`` (the position time_attention() times, so traffic and
    bytes_per_launch describe the same launch)."""
    from lit_gpt import ops

    C, N, copies = 4096, 11008, 24
    dev = torch.device("cuda")
    sets = []
    for _ in range(copies):
        q1, s1 = ops.quantize(torch.randn(N, C, device=dev) * 0.02, 0, 128)
        q2, s2 = ops.quantize(torch.randn(N, C, device=dev) * 0.02, 0, 128)
        sets.append((q1, s1, q2, s2))
    x = torch.randn(C, device=dev).to(torch.bfloat16)
    nw = torch.ones(C, device=dev).to(torch.bfloat16)
    out = torch.empty(N, dtype=torch.bfloat16, device=dev)
    torch.cuda.synchronize()
    for q1, s1, q2, s2 in sets:
        ops.q4_gemv_swiglu(x, q1, s1, q2, s2, N, C, 128, 0, norm_weight=nw, out=out)
    torch.cuda.synchronize()
    del sets
    # the decode attention over 24 distinct layers' K/V caches at the bench's last position (0.9 GB)
    H = G = 32
    hs, S = 128, max(PROMPT_LEN + 256, att_pos + 2)
    pos = torch.tensor([att_pos], device=dev)
    cos, sin = torch.ones(S, hs, device=dev), torch.zeros(S, hs, device=dev)
    qkv = torch.randn(1, (H + 2 * G) * hs, device=dev).to(torch.bfloat16)
    splits = ops.decode_splits(G, H // G, hs, S)
    ws = ops.AttentionWorkspace(1, H, G, hs, splits, dev)
    caches = [(torch.randn(G, S, hs, device=dev).to(torch.bfloat16), torch.randn(G, S, hs, device=dev).to(torch.bfloat16))
              for _ in range(copies)]
    torch.cuda.synchronize()
    for kc, vc in caches:
        ops.attention_decode_fused(qkv, kc, vc, pos, pos, cos, sin, H, G, hs, hs, hs ** -0.5, splits, workspace=ws)
    torch.cuda.synchronize()


def measure_traffic(att_pos: int, timeout_s: float = 240.0):
    """HBM bytes per launch of the dominant kernel from the PMC counters, collected as MI355X_MICROARCH.md's HBM
    section prescribes: FETCH_SIZE (KiB, TCC_EA0_RDREQ x 64 B) in its own rocprofv3 pass, doubled (gfx950 tallies
    128-B requests of a 16-B/lane streaming read at 64 B). Runs in a child process started BEFORE this process
    touches the GPU. Returns {"gemv" | "attention": (bytes per launch or None, note)}."""
    import csv
    import shutil
    import statistics
    import subprocess
    import tempfile

    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not Path(exe).exists():
        return None, "rocprofv3 not found"
    out = Path(tempfile.mkdtemp(prefix="lga_pmc_"))
    cmd = [exe, "--pmc", "FETCH_SIZE", "--output-format", "csv", "-d", str(out), "-o", "pmc", "--",
           sys.executable, str(Path(__file__).resolve()), "--pmc-child", "--pmc-pos", str(att_pos)]
    try:
        subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=timeout_s, check=True)
        files = list(out.rglob("*counter_collection.csv"))
        rows = [r for f in files for r in csv.DictReader(open(f)) if r.get("Counter_Name") == "FETCH_SIZE"]
        res = {}
        for key, pat in (("gemv", "gemv_q4"), ("attention", "attn_kernel")):
            vals = [float(r["Counter_Value"]) for r in rows if pat in r.get("Kernel_Name", "")]
            if not vals:
                res[key] = (None, f"no FETCH_SIZE rows for {pat}")
                continue
            kib = statistics.median(vals)
            res[key] = (2.0 * kib * 1024.0, f"median FETCH_SIZE {kib:.0f} KiB over {len(vals)} launches, x2 (gfx950)")
        return res
    except Exception as e:  # traffic is diagnostic; never lose the bench line over it
        return {k: (None, f"pmc pass failed: {type(e).__name__}") for k in ("gemv", "attention")}
    finally:
        shutil.rmtree(out, ignore_errors=True)


def cpu_baseline(cfg, threads: int, seconds: float = 15.0):
    """The oracle (CPU restatement of the reference's bf16 decode math) on a bounded sample: 2 of the 32 blocks
    at full Llama-2-7B width + lm_head, KV context 2048, repeated decode steps; per-token time extrapolated to
    all 32 blocks."""
    from oracle import model as om

    torch.set_num_threads(threads)
    small = type(cfg)(**{**{k: getattr(cfg, k) for k in cfg.__dataclass_fields__}, "n_layer": 2})
    g = torch.Generator().manual_seed(0)
    sd = {}
    from oracle import synth

    for name, shape, kind in synth.param_shapes(small):
        if kind == "normal":
            sd[name] = (torch.randn(shape, generator=g) * 0.02).numpy()
        else:
            sd[name] = torch.ones(shape).numpy() if kind == "ones" else torch.zeros(shape).numpy()
    m = om.OracleGPT(small, sd, dtype=torch.bfloat16)
    del sd
    S = PROMPT_LEN + 64
    m.set_kv_cache(S)
    for i in range(2):  # fill a 2048-long context cheaply (random K/V; attention cost is what matters)
        m.cache.write(i, torch.arange(PROMPT_LEN),
                      torch.randn(small.n_query_groups, PROMPT_LEN, small.head_size).bfloat16(),
                      torch.randn(small.n_query_groups, PROMPT_LEN, small.head_size).bfloat16())
    tok = torch.tensor([1])
    with torch.inference_mode():
        m.forward(tok, torch.tensor([PROMPT_LEN]))  # warm-up
        t_layers, t_head, n = 0.0, 0.0, 0
        t_start = time.perf_counter()
        pos = PROMPT_LEN + 1
        while time.perf_counter() - t_start < seconds and pos < S:
            t0 = time.perf_counter()
            m.forward(tok, torch.tensor([pos]))
            t_layers += time.perf_counter() - t0
            n += 1
            pos += 1
        # lm_head + final norm share of one forward (measured separately so the 2->32 block scaling is exact)
        x = torch.randn(1, small.n_embd).bfloat16()
        t0 = time.perf_counter()
        for _ in range(n):
            m._lin("lm_head", m._norm("transformer.ln_f", x))
        t_head = (time.perf_counter() - t0) / n
    per_fwd = t_layers / n
    per_block = (per_fwd - t_head) / 2
    per_token = per_block * cfg.n_layer + t_head
    return {"value": round(1.0 / per_token, 3), "unit": "tokens/s", "cores": threads, "kind": "port",
            "sample": f"oracle bf16 decode, {n} steps at context ~{PROMPT_LEN} over 2 of {cfg.n_layer} "
                      f"Llama-2-7B blocks + lm_head, extrapolated to {cfg.n_layer} blocks "
                      f"({per_token * 1e3:.1f} ms/token)"}


def time_sampled_decode(model, first, T: int, warmup: int, steps: int, barrier, world: int):
    """The reference's default sampling (generate/base.py:102-103: top_k 200, temperature 0.8) as captured decode
    steps: the same positions as the greedy timed region, the argmax replaced by the fused top-k + softmax +
    inverse-CDF sampler (ops.sample_topk inside DecodeGraph). Also the sampler launch alone on the step's logits."""
    from generate.base import SamplerRNG
    from lit_gpt import ops
    from lit_gpt.runtime import DecodeGraph

    dev = first.device
    torch.manual_seed(1234)
    rng = SamplerRNG(dev)
    dg = DecodeGraph(model, first, T, chunk=CHUNK, temperature=0.8, top_k=200, rng=rng)

    def run(n):
        done = 0
        while n - done >= CHUNK > 1:
            dg.steps()
            done += CHUNK
        for _ in range(n - done):
            dg.step()

    run(warmup)
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    logits = model(dg.token, dg.pos, last_token_only=True).reshape(-1).contiguous()
    counter = torch.zeros(1, dtype=torch.int64, device=dev)
    out = torch.zeros(1, dtype=torch.int64, device=dev)
    for _ in range(5):
        ops.sample_topk(logits, 200, 0.8, seed=rng.seed, counter=counter, out_idx=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100):
        ops.sample_topk(logits, 200, 0.8, seed=rng.seed, counter=counter, out_idx=out)
    e1.record()
    torch.cuda.synchronize()
    return {"top_k": 200, "temperature": 0.8, "tokens_per_s": round(steps / elapsed, 2),
            "ms_per_step": round(elapsed / steps * 1e3, 4), "sampler_us": round(e0.elapsed_time(e1) * 10, 2),
            "note": "generate/base.py's default sampling, captured: the greedy run's positions with the argmax "
                    "replaced by lga_sample_topk (top-k radix select, bf16 softmax, inverse CDF on a counter-based "
                    "uniform, embedding row gather); sampler_us = that launch alone on one step's logits"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: the eager capture step (p = 2048) + 14 warm-up + 240 timed steps = the 255 decode steps of
    # SURVEY §8d (p = 2048 ... 2302)
    ap.add_argument("--steps", type=int, default=240)
    ap.add_argument("--warmup", type=int, default=14)
    ap.add_argument("--quantize", default="int4-g128",
                    help="4-bit mode, or 'bf16' for unquantized weights (BASELINE config 2)")
    ap.add_argument("--model", default=MODEL, help="lit_gpt Config name (default: the headline Llama-2-7B)")
    ap.add_argument("--prompt_len", type=int, default=PROMPT_LEN)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-sample", action="store_true",
                    help="skip the sampled-decode line (top_k 200, temperature 0.8: generate/base.py's defaults)")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC pass for roofline.traffic")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--pmc-pos", type=int, default=PROMPT_LEN + 254, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.pmc_child:
        return pmc_child(args.pmc_pos)
    traffic = {k: (None, "skipped") for k in ("gemv", "attention")}
    under_profiler = any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ)
    headline = args.model == MODEL and args.quantize == "int4-g128"
    dense = args.quantize in ("bf16", "none")
    if int(os.environ.get("WORLD_SIZE", "1")) == 1 and not args.no_traffic and not under_profiler and headline:
        # before this process initialises the GPU; the attention at the position time_attention() uses below
        traffic = measure_traffic(args.prompt_len + args.warmup + args.steps)

    import torch.distributed as dist

    from generate import tp as gtp
    from generate.base import build_model
    from lit_gpt import Config
    from lit_gpt.runtime import DecodeGraph

    fabric = gtp.init_distributed()
    world, rank = fabric.world_size, fabric.global_rank
    dev = torch.device("cuda", torch.cuda.current_device())
    cfg = Config.from_name(args.model)
    T = args.prompt_len
    max_seq = T + args.warmup + args.steps + 2
    t0 = time.perf_counter()
    from functools import partial

    model = build_model(cfg, quantize=None if dense else args.quantize, device=dev, max_seq_length=max_seq,
                        fabric=fabric if world > 1 else None, prefill_rows=T)
    load_s = time.perf_counter() - t0
    g = torch.Generator(device="cpu").manual_seed(1234)
    prompt = torch.randint(0, cfg.vocab_size, (T,), generator=g, dtype=torch.int32).to(dev)

    def barrier():
        if world > 1:
            dist.barrier()

    with torch.inference_mode():
        # prefill (reference-style tok/s includes it; reported separately)
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        logits = model(prompt.view(1, -1), torch.arange(T, device=dev), last_token_only=True)
        from lit_gpt import ops

        first = ops.argmax(logits.reshape(-1)).to(torch.int32)
        torch.cuda.synchronize()
        prefill_s = time.perf_counter() - t0
        # warm prefill for the MFMA rate (rewrites cache rows 0..T-1 with the same values; the cold first call
        # above also pays code-object loading and is what reference-style tok/s counts)
        barrier()
        t0 = time.perf_counter()
        model(prompt.view(1, -1), torch.arange(T, device=dev), last_token_only=True)
        torch.cuda.synchronize()
        prefill_warm_s = time.perf_counter() - t0
        use_graph = not args.no_graph
        graph_note = None
        if use_graph:
            try:  # first decode step runs eagerly, then the step (and CHUNK steps as one graph) is captured
                dg = DecodeGraph(model, first, T, chunk=CHUNK)
            except Exception as e:  # e.g. a collective backend that cannot be captured: time the eager loop
                use_graph, graph_note = False, f"graph capture failed ({type(e).__name__}); eager steps"
                torch.cuda.synchronize()
                barrier()
        if use_graph:
            def step():
                dg.step()
        else:
            from generate.base import next_token

            tok = first.view(1, 1)
            pos = torch.tensor([T], device=dev)

            def step():
                nonlocal tok
                tok = next_token(model, pos, tok.view(1, 1), temperature=0.0)
                pos.add_(1)
        def run(n, marks=None):  # n decode steps: whole CHUNK-step graph launches, then single steps
            done = 0
            while use_graph and n - done >= CHUNK > 1:
                dg.steps()
                done += CHUNK
                if marks is not None:  # GPU-side marks between launches (the step-time spread; no host sync)
                    ev = torch.cuda.Event(enable_timing=True)
                    ev.record()
                    marks.append(ev)
            for _ in range(n - done):
                step()

        run(args.warmup)
        torch.cuda.synchronize()
        barrier()
        marks = []
        t0 = time.perf_counter()
        run(args.steps, marks)
        torch.cuda.synchronize()
        barrier()
        elapsed = time.perf_counter() - t0
        launch_ms = [a.elapsed_time(b) / CHUNK for a, b in zip(marks, marks[1:])]
        gtp.comm.check_errors()  # TP: a timed-out xGMI all-reduce voids the run (raises on every rank)
        if world > 1:
            t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        tok_s = args.steps / elapsed
        ms_step = elapsed / args.steps * 1e3
        avg_ms, kbytes = time_dominant_kernel(model)
        att_ms, att_bytes = time_attention(model, T + args.warmup + args.steps)
        sampled = None
        from generate.base import graph_sampling

        if use_graph and not args.no_sample and graph_sampling(model, 0.8, 200):
            sampled = time_sampled_decode(model, first, T, args.warmup, args.steps, barrier, world)

    cfg_full = Config.from_name(args.model)
    pf_flops = prefill_flops(cfg_full, T, tp=world)
    mean_pos = T + args.warmup + 1 + (args.steps - 1) / 2
    step_bytes = algorithmic_bytes_per_token(cfg_full, mean_pos, tp=world, dense=dense)
    step_gbs = step_bytes * tok_s / 1e9
    kern_gbs = kbytes / (avg_ms * 1e-3) / 1e9
    gemv_line = {"bound": "hbm", "kernel": (
                 "gemv_bf16_kernel<.., DUAL> (RMSNorm + fc_1/fc_2 bf16 GEMV + SwiGLU of one block)" if dense else
                 DOMINANT if not cfg._mlp_class == "LLaMAMoE" else
                 "gemv_q4_kernel<.., DUAL> routed (RMSNorm + fc_1/fc_2 of 2 experts + SwiGLU of one block)"),
                 "achieved": round(kern_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": round(kern_gbs / HBM_PEAK_GBS, 4),
                 "traffic": None if traffic["gemv"][0] is None else int(traffic["gemv"][0]),
                 "traffic_note": traffic["gemv"][1],
                 "bytes_per_launch": int(kbytes), "avg_launch_us": round(avg_ms * 1e3, 2),
                 "us_per_step": round(avg_ms * 1e3 * cfg.n_layer, 1)}
    att_line = None if att_ms is None else {
        "bound": "hbm", "kernel": "attn_kernel<..,FUSED> (RoPE + KV append + split decode attention of one block)",
        "achieved": round(att_bytes / (att_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(att_bytes / (att_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "bytes_per_launch": int(att_bytes),
        "traffic": None if traffic["attention"][0] is None else int(traffic["attention"][0]),
        "traffic_note": traffic["attention"][1], "avg_launch_us": round(att_ms * 1e3, 2),
        "us_per_step": round(att_ms * 1e3 * cfg.n_layer, 1), "position": T + args.warmup + args.steps}
    # the roofline object reports the kernel with the most device time per decode step (one launch per block
    # each); the other one rides along as roofline_secondary
    lines = sorted([l for l in (gemv_line, att_line) if l is not None], key=lambda l: -l["us_per_step"])
    for l in lines:
        l["note"] = ("the largest per-step kernel (most us per decode step)" if l is lines[0] else
                     "second-largest per-step kernel")
    result = {
        "metric": ("decode tokens/s/GPU (Llama-2-7B int4, seq=2048) + % HBM roofline" if headline else
                   f"decode tokens/s/GPU ({args.model} {args.quantize}, seq={T}) + % HBM roofline"),
        "value": round(tok_s, 2),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (random-init N(0,0.02) weights, uniform random prompt ids)",
        "config": {"workload": f"{args.model} single-stream greedy decode after a {T}-token prefill",
                   "weights": args.quantize, "prompt_len": T, "decode_positions": [T + args.warmup + 1,
                                                                                   T + args.warmup + args.steps],
                   "global_batch": 1, "seq_len": T, "parallelism": f"tp{world}",
                   "graph": use_graph, "steps_per_graph_launch": CHUNK if use_graph else 0,
                   **({"graph_note": graph_note} if graph_note else {}),
                   **({"allreduce": (f"xgmi one-shot, fused GEMV protocol {gtp.comm.get_default().protocol}" +
                                     ("" if gtp.comm.get_default().fused_ok else
                                                        f" (fused GEMV form off: {gtp.comm.get_default().fused_fallback})"))
                       if gtp.comm.get_default() is not None else
                       f"rccl ({gtp.comm.fallback_reason or 'LGA_TP_ALLREDUCE=rccl'})"} if world > 1 else {})},
        "roofline": lines[0],
        "roofline_secondary": lines[1] if len(lines) > 1 else None,
        "step_roofline": {"bytes_per_token": int(step_bytes), "achieved": round(step_gbs, 1),
                          "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(step_gbs / HBM_PEAK_GBS, 4),
                          "roofline_tokens_per_s": round(HBM_PEAK_GBS * 1e9 / step_bytes, 1)},
        "prefill_s": round(prefill_s, 4),
        "prefill_roofline": {"bound": "mfma", "flops": pf_flops,
                             "seconds": round(prefill_s, 5),
                             "achieved": round(pf_flops / prefill_s / 1e12, 1),
                             "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                             "frac": round(pf_flops / prefill_s / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4),
                             "warm_seconds": round(prefill_warm_s, 5),
                             "warm_achieved": round(pf_flops / prefill_warm_s / 1e12, 1),
                             "warm_frac": round(pf_flops / prefill_warm_s / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4),
                             "note": "seconds / frac: the FIRST (cold) prefill of the process, wall clock, the one "
                                     "reference-style tok/s counts; warm_*: the same prompt run a second time; every "
                                     "Linear's int4 weights dequantized inside the GEMM, flash attention, norms"},
        "step_time_ms": None if len(launch_ms) < 2 else {
            "p50": round(float(np.percentile(launch_ms, 50)), 4), "p95": round(float(np.percentile(launch_ms, 95)), 4),
            "max": round(max(launch_ms), 4), "launches": len(launch_ms),
            "note": f"per {CHUNK}-step graph launch / {CHUNK}, GPU events between the timed launches"},
        "reference_style_tokens_per_s": round((args.steps + args.warmup + 1) / (prefill_s + elapsed * (
            args.steps + args.warmup + 1) / args.steps), 2),
        "load_s": round(load_s, 2),
        "sampled_decode": sampled,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and headline:
        # the reference's CPU path on all the host cores this process may run on — the affinity set,
        # capped by the CPU share the host grants the job (OMP_NUM_THREADS: 16 per GPU on the MI355X pool, whose
        # affinity mask shows the whole machine)
        threads = len(os.sched_getaffinity(0)) or os.cpu_count() or 1
        if os.environ.get("OMP_NUM_THREADS", "").isdigit():
            threads = min(threads, int(os.environ["OMP_NUM_THREADS"]))
        try:
            result["cpu_baseline"] = cpu_baseline(cfg_full, threads, args.cpu_seconds)
        except Exception as e:  # the baseline is reported, never the target: do not lose the GPU number
            result["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
