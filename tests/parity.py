"""Logit parity bounds shared by the GPU end-to-end tests (test_gpu_geometry.py, test_gpu_tp.py).

Both sides of a comparison compute in bf16 with fp32 accumulation, but in different orders and (inside fused
kernels) with different intermediate rounding points, so "within x % of the bf16 reference" is only meaningful
relative to how far bf16 itself is from exact arithmetic. Every check therefore takes two references computed on the
SAME weights and the SAME token stream:

* ``ref_bf16`` — the reference's ``--precision bf16-true`` path (the oracle in bf16, or the reference's own bf16
  logits from a fixture);
* ``ref_exact`` — the same math in float64 (oracle) or float32 (reference fixture): the exact-arithmetic stand-in.

and asserts, per step (relative to the logit scale max |ref_exact| and the RMS logit):

* accuracy — the product's distance to ``ref_exact`` is at most ``ACC_FACTOR`` x the reference-bf16 path's own
  distance to it, plus ``ACC_SLACK`` (the product is as accurate as the reference running in bf16), max and rms;
* agreement — the product is within ``AGREE_REL`` of ``ref_bf16`` (max and rms): two independent bf16 evaluations
  land about sqrt(2) x the floor apart; the floor at Llama-2-7B width is 1.6-1.9 % (tools/bf16_noise_floor.py);
* tokens — the product's argmax equals ``ref_exact``'s wherever that top-1/top-2 margin exceeds 4 x the product's
  observed max error.
"""

from __future__ import annotations

import math

import numpy as np

ACC_FACTOR = 1.25
ACC_SLACK = 0.0025
AGREE_REL = 0.03


def rel_err(got, exp):
    got = np.asarray(_np(got), dtype=np.float64)
    exp = np.asarray(_np(exp), dtype=np.float64)
    err = np.abs(got - exp)
    return (float(err.max() / np.abs(exp).max()), math.sqrt(float((err ** 2).mean()) / float((exp ** 2).mean())),
            float(err.max()))


def check_step(got, ref_bf16, ref_exact, tag: str, agree: float = AGREE_REL) -> float:
    """Assert the module's bounds for one step's logits (1-D arrays or tensors); returns the product's max error
    relative to the exact reference."""
    got, ref_bf16, ref_exact = (np.asarray(_np(a), dtype=np.float64) for a in (got, ref_bf16, ref_exact))
    g_max, g_rms, g_abs = rel_err(got, ref_exact)
    r_max, r_rms, _ = rel_err(ref_bf16, ref_exact)
    a_max, a_rms, _ = rel_err(got, ref_bf16)
    order = np.argsort(ref_exact)
    margin = float(ref_exact[order[-1]] - ref_exact[order[-2]])
    print(f"{tag}: vs exact max {g_max:.3%} rms {g_rms:.3%} (bf16 reference: {r_max:.3%} / {r_rms:.3%}); "
          f"vs bf16 reference max {a_max:.3%} rms {a_rms:.3%}; margin {margin:.3f}")
    assert g_max <= ACC_FACTOR * r_max + ACC_SLACK, f"{tag}: max error vs exact {g_max:.3%} (bf16 ref {r_max:.3%})"
    assert g_rms <= ACC_FACTOR * r_rms + ACC_SLACK, f"{tag}: rms error vs exact {g_rms:.3%} (bf16 ref {r_rms:.3%})"
    assert a_max <= agree and a_rms <= agree, f"{tag}: {a_max:.3%} / {a_rms:.3%} from the bf16 reference"
    if margin > 4 * g_abs:
        assert int(np.argmax(got)) == int(order[-1]), f"{tag}: greedy token differs from the reference"
    return g_max


def _np(a):
    if hasattr(a, "detach"):
        return a.detach().double().cpu().numpy()
    return a
