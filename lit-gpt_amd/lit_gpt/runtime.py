"""Decode-step executor: one HIP graph per greedy decode step.

The reference gets launch-overhead relief from ``torch.compile(next_token, mode="reduce-overhead")``
(generate/base.py:161-166), i.e. CUDA graphs over Inductor/Triton kernels. Here the step is already a short
chain of hand-written HIP kernels (per layer: fused RMSNorm+qkv GEMV, RoPE+KV append, split attention +
combine, proj GEMV+residual, fused RMSNorm+SwiGLU GEMV, down GEMV+residual; then RMSNorm+lm_head GEMV and
argmax). ``DecodeGraph`` captures that chain once with static input buffers — the token id and ``input_pos``
live on the device, the argmax kernel writes the next token and advances ``input_pos`` — so a decode step is a
single ``hipGraphLaunch`` with no host<->device synchronisation.
"""

from __future__ import annotations

from typing import Optional

import torch

from lit_gpt import ops


class DecodeGraph:
    def __init__(self, model, first_token: torch.Tensor, first_pos: int) -> None:
        """Runs one real decode step eagerly (token ``first_token`` at position ``first_pos``) to warm up, then
        captures the step. Afterwards ``self.token`` holds the newest token and ``self.pos`` its position."""
        dev = first_token.device
        self.model = model
        self.token = first_token.reshape(1, 1).to(torch.int32).clone()
        self.pos = torch.tensor([first_pos], dtype=torch.int64, device=dev)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self._step_eager()
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._step_body()
        self.graph = g

    def _step_body(self) -> None:
        logits = self.model(self.token, self.pos, last_token_only=True)
        ops.argmax(logits.reshape(-1), token_out=self.token.view(-1), pos_inout=self.pos)

    def _step_eager(self) -> None:
        self._step_body()

    def step(self) -> torch.Tensor:
        """One decode step; returns the (device) token buffer holding the new token."""
        self.graph.replay()
        return self.token
