"""RMSNorm module (reference lit_gpt/rmsnorm.py:6-28) backed by the ``lga_rmsnorm`` HIP kernel."""

from __future__ import annotations

import torch
import torch.nn as nn

from lit_gpt import ops


def _gpu_only(what: str) -> None:
    raise RuntimeError(f"{what}: this build computes on the MI355X only (no CPU path); move the model to 'cuda'")


class RMSNorm(nn.Module):
    """lit_gpt/rmsnorm.py:6-28 on the GPU (``lga_rmsnorm``): fp32 math, one cast back to bf16."""

    def __init__(self, size: int, dim: int = -1, eps: float = 1e-5) -> None:
        super().__init__()
        self.weight = nn.Parameter(torch.ones(size))
        self.eps = eps
        self.dim = dim

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:
            _gpu_only("RMSNorm")
        return ops.rmsnorm(x.contiguous(), self.weight, self.eps)

    def reset_parameters(self) -> None:
        torch.nn.init.ones_(self.weight)
