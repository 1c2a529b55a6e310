"""Tensor-parallel sharding restatement — TEST INFRASTRUCTURE ONLY (oracle/__init__.py).

generate/tp.py:28-45 (``tensor_parallel_linear``): colwise = split dim 0 (out_features), rowwise =
split dim 1 (in_features), ``torch.tensor_split(W, world, dim)[rank]``; the bias is split only for
colwise (rowwise bias is kept whole, so the all-reduce adds it ``world`` times: reference bug).
"""

from __future__ import annotations

from typing import Optional, Tuple

import numpy as np


def shard_linear(w: np.ndarray, b: Optional[np.ndarray], style: str, world: int, rank: int
                 ) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    dim = {"colwise": 0, "rowwise": 1}[style]
    if w.shape[dim] % world:
        attr = "out_features" if dim == 0 else "in_features"
        raise ValueError(f"This linear's {attr} value ({w.shape[dim]}) is not evenly divisible by the world size ({world})")
    ws = np.array_split(w, world, axis=dim)[rank]
    bs = b if (b is None or dim == 1) else np.array_split(b, world)[rank]
    return np.ascontiguousarray(ws), bs
