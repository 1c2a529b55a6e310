"""Decode-step executor: one HIP graph per decode step (greedy, or top-k sampling at temperature > 0).

The reference gets launch-overhead relief from ``torch.compile(next_token, mode="reduce-overhead")``
(generate/base.py:161-166), i.e. CUDA graphs over Inductor/Triton kernels. Here the step is already a short
chain of hand-written HIP kernels (per layer: fused RMSNorm+qkv GEMV, RoPE+KV append, split attention +
combine, proj GEMV+residual, fused RMSNorm+SwiGLU GEMV, down GEMV+residual; then RMSNorm+lm_head GEMV and
argmax). ``DecodeGraph`` captures that chain once with static input buffers — the token id and ``input_pos``
live on the device, the argmax kernel writes the next token, advances ``input_pos`` and gathers the token's
embedding row for the next step (so the step has no embedding launch) — so a decode step is a single
``hipGraphLaunch`` with no host<->device synchronisation (or, with ``chunk``, several steps are).
"""

from __future__ import annotations

import os
from typing import Optional

import torch

from lit_gpt import ops

class DecodeGraph:
    def __init__(self, model, first_token: torch.Tensor, first_pos: int, chunk: int = 1, *,
                 temperature: float = 0.0, top_k: Optional[int] = None, rng=None) -> None:
        """Runs one real decode step eagerly (token ``first_token`` at position ``first_pos``) to warm up, then
        captures the step. Afterwards ``self.token`` holds the newest token and ``self.pos`` its position.
        ``chunk`` > 1 also captures ``chunk`` consecutive steps as one graph (``steps()``): the argmax of step i
        writes its token into ``self.history[i]`` as well, and one launch replaces ``chunk`` (≈9 us of
        graph-launch gap per step on MI355X, profiles/r02b_*). ``temperature`` > 0 replaces the argmax with the
        fused top-k sampler (ops.sample_topk, ``top_k`` 1..1024, RNG state ``rng``: generate.base.SamplerRNG)."""
        dev = first_token.device
        self.model = model
        self.temperature, self.top_k, self.rng = float(temperature), top_k, rng
        if self.temperature > 0.0 and (rng is None or top_k is None or not 1 <= top_k <= ops.MAX_TOP_K):
            raise ValueError("DecodeGraph: sampling needs top_k in [1, 1024] and an rng (generate.base.SamplerRNG)")
        self.token = first_token.reshape(1, 1).to(torch.int32).clone()
        self.pos = torch.tensor([first_pos], dtype=torch.int64, device=dev)
        self.chunk = max(1, int(chunk))
        self.history = torch.zeros(self.chunk, dtype=torch.int64, device=dev)
        # the argmax launch also gathers the new token's embedding row (ops.argmax_embed) into x_emb, which the
        # next step's forward takes instead of running its own embedding launch
        wte = model.transformer.wte.weight
        self.fuse_embedding = (wte.is_cuda and wte.dtype == torch.bfloat16 and wte.is_contiguous()
                               and wte.shape[1] % 8 == 0)
        self.x_emb = torch.empty(wte.shape[1], dtype=torch.bfloat16, device=dev) if self.fuse_embedding else None
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.chunk_graph: Optional[torch.cuda.CUDAGraph] = None
        self._step_eager()
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._step_body()
        self.graph = g
        if self.chunk > 1:
            gc = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gc):
                for i in range(self.chunk):
                    self._step_body(self.history[i:i + 1])
            self.chunk_graph = gc

    # greedy steps run ln_f + lm_head + argmax + the next embedding row as ONE launch (ops.q4_gemv_argmax_embed)
    # where the head is a 4-bit Linear it covers; False keeps lm_head GEMV + argmax_embed (bit-identical)
    fuse_head = os.environ.get("LGA_FUSE_HEAD", "1") != "0"

    def _step_body(self, idx_out: Optional[torch.Tensor] = None, embedded: bool = True) -> None:
        fuse = self.fuse_embedding
        model = self.model
        ln = model.transformer.ln_f
        if (self.temperature == 0.0 and fuse and self.fuse_head and ops.head_argmax_supported(model.lm_head)
                and type(ln).__name__ == "RMSNorm" and not model.lm_head._forward_hooks):
            h = model(self.token, self.pos, last_token_only=True, embedded=self.x_emb if embedded else None,
                      hidden_only=True).reshape(-1)
            if getattr(self, "_head_ws", None) is None:
                self._head_ws = ops.HeadWorkspace(model.lm_head.out_features, model.lm_head.in_features, h.device)
                self.logits = torch.empty(model.lm_head.out_features, dtype=torch.bfloat16, device=h.device)
            ops.q4_gemv_argmax_embed(h, model.lm_head, self._head_ws, norm_weight=ln.weight, eps=ln.eps,
                                     table=model.transformer.wte.weight, emb_out=self.x_emb, logits=self.logits,
                                     out_idx=idx_out, token_out=self.token.view(-1), pos_inout=self.pos)
            return
        logits = model(self.token, self.pos, last_token_only=True,
                       embedded=self.x_emb if (fuse and embedded) else None).reshape(-1)
        table = model.transformer.wte.weight if fuse else None
        if self.temperature > 0.0:
            ops.sample_topk(logits, self.top_k, self.temperature, seed=self.rng.seed, counter=self.rng.counter,
                            out_idx=idx_out, token_out=self.token.view(-1), pos_inout=self.pos, table=table,
                            emb_out=self.x_emb)
        elif fuse:
            ops.argmax_embed(logits, table, self.x_emb, out_idx=idx_out, token_out=self.token.view(-1),
                             pos_inout=self.pos)
        else:
            ops.argmax(logits, out_idx=idx_out, token_out=self.token.view(-1), pos_inout=self.pos)

    def _step_eager(self) -> None:
        self._step_body(embedded=False)  # embeds first_token itself; its argmax leaves x_emb for the graphs

    def step(self) -> torch.Tensor:
        """One decode step; returns the (device) token buffer holding the new token."""
        self.graph.replay()
        return self.token

    def steps(self) -> torch.Tensor:
        """``chunk`` decode steps in one graph launch; returns the (device, int64) buffer of their tokens."""
        if self.chunk_graph is None:
            raise RuntimeError("DecodeGraph was built with chunk=1")
        self.chunk_graph.replay()
        return self.history
