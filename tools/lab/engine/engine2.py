"""LAB: persistent decode engine, version 2 (``lga_decode_engine`` of tools/lab/engine/engine2.hip, built into
tools/_lab/liblga_engine2.so by ``make -C lit-gpt_amd/csrc lab-engine2``): register-streaming compute waves, gather
waves that never stream, a CU-local qkv -> attention edge (design notes at the top of engine2.hip). Same C-ABI as
version 1 (tools/lab/engine/engine.h) plus ``lga_engine_layout`` for the tests.

The reference runs a decode step as ``next_token`` -> ``GPT.forward`` -> every ``Block.forward`` -> ``ln_f`` ->
``lm_head`` -> ``sample`` (reference generate/base.py:44-47,87-92; lit_gpt/model.py:499-519,572-593), ~50 kernels
per block. The per-op path of this build (model.py + runtime.DecodeGraph) replays that chain as 160 hand-written
kernels per step in one HIP graph; ``DecodeEngine`` runs the same math as ONE persistent kernel whose per-CU
loader wave streams the weights and K/V rows ahead of the compute across op boundaries (design: csrc/engine.hip,
DESIGN.md §4.6). GEMV outputs are bit-identical to the per-op kernels'; attention merges its key splits in a
different order (same math, fp32 online softmax).

Scope (``lga_engine_check``): Llama-family blocks (RMSNorm, LLaMAMLP, no bias), int4-g weights of one group size in
every Linear incl. lm_head, head_size == rope_n_elem == 128, q_per_kv 1, Llama-2-7B-class widths, no tensor
parallelism. Everything else keeps the per-op path (``DecodeEngine.supported`` returns the reason).
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path
from typing import Optional, Tuple

import torch

from lit_gpt import ops

LAB_LIB = Path(os.environ.get("LGA_ENGINE2_LIB", Path(__file__).resolve().parents[2] / "_lab" / "liblga_engine2.so"))
_elib: Optional[ctypes.CDLL] = None


def engine_library() -> ctypes.CDLL:
    """The lab library (product objects + the engine), loaded once with the engine's signatures."""
    global _elib
    if _elib is None:
        if not LAB_LIB.is_file():
            raise ops.NativeLibraryError(f"lab engine library not found at {LAB_LIB}: make -C lit-gpt_amd/csrc lab-engine2")
        lib = ctypes.CDLL(str(LAB_LIB))
        P, I = ctypes.c_void_p, ctypes.c_int
        sig = {"lga_engine_check": ([P], I), "lga_engine_scratch_bytes": ([P], ctypes.c_size_t),
               "lga_engine_x0": ([P, P], ctypes.c_void_p), "lga_engine_reset": ([P, P, P], I),
               "lga_engine_error": ([P, P, P], I),
               "lga_decode_engine": ([P] * 13 + [I, P], I), "lga_last_error_string": ([], ctypes.c_char_p),
               "lga_engine_layout": ([P, P], I)}
        for name, (args, res) in sig.items():
            fn = getattr(lib, name)
            fn.argtypes, fn.restype = args, res
        _elib = lib
    return _elib


def _check(rc: int) -> None:
    if rc != 0:
        raise RuntimeError(f"engine error {rc}: {engine_library().lga_last_error_string().decode()}")


class EngineLayer(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("qkv_w", "qkv_s", "o_w", "o_s", "fc1_w", "fc1_s", "fc2_w", "fc2_s",
                                               "dn_w", "dn_s", "norm1", "norm2", "k_cache", "v_cache")]


class EngineGeom(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("n_layer", "n_embd", "n_head", "n_query_groups", "head_size",
                                            "intermediate", "vocab", "max_seq", "group", "fmt", "rope_rows",
                                            "n_cu")] + [("norm_eps", ctypes.c_float), ("attn_scale", ctypes.c_float)]


class EngineTimeout(RuntimeError):
    """A launch of the engine gave up waiting (a CU never arrived): its outputs are invalid and the engine state
    was reset."""


def _why_not(model) -> Optional[str]:
    from lit_gpt.model import LLaMAMLP
    from lit_gpt.quantize import QuantLinear
    from lit_gpt.rmsnorm import RMSNorm

    c = model.config
    if not isinstance(model.lm_head, QuantLinear):
        return "lm_head is not a 4-bit QuantLinear"
    lins = [model.lm_head]
    for b in model.transformer.h:
        if not isinstance(b.norm_1, RMSNorm) or not isinstance(b.norm_2, RMSNorm) or not isinstance(b.mlp, LLaMAMLP):
            return "not a Llama-family block"
        if c.parallel_residual or c.shared_attention_norm:
            return "parallel residual / shared norm"
        mods = (b.attn.attn, b.attn.proj, b.mlp.fc_1, b.mlp.fc_2, b.mlp.proj)
        if any(not isinstance(m, QuantLinear) or m.bias is not None for m in mods):
            return "a block Linear is not a bias-free QuantLinear"
        if any(m._forward_hooks or m._forward_pre_hooks for m in (b, b.attn, b.mlp) + mods):
            return "forward hooks (tensor parallelism) need the per-op path"
        if b.attn.kv_cache is None:
            return "no KV cache"
        lins += list(mods)
    if len({(m.fmt, m.group) for m in lins}) != 1:
        return "Linears of different 4-bit formats"
    if c.rope_n_elem != c.head_size:
        return "partial rotary"
    if not isinstance(model.transformer.ln_f, RMSNorm):
        return "ln_f is not RMSNorm"
    wte = model.transformer.wte.weight
    if not wte.is_cuda or wte.dtype != torch.bfloat16 or not wte.is_contiguous():
        return "embedding table is not a contiguous bf16 GPU tensor"
    return None


class DecodeEngine:
    """Owns the device-side layer table and the engine scratch for one model; ``step`` launches one decode step
    (graph-capturable: every argument is a fixed device pointer)."""

    def __init__(self, model, n_cu: Optional[int] = None) -> None:
        why = _why_not(model)
        if why is not None:
            raise NotImplementedError(f"DecodeEngine: {why}")
        self.model = model
        c = model.config
        blocks = model.transformer.h
        dev = model.transformer.wte.weight.device
        self.device = dev
        kv = blocks[0].attn.kv_cache
        cos, sin = model._rope_tables()
        self.cos, self.sin = cos.contiguous(), sin.contiguous()
        lm = model.lm_head
        self.geom = EngineGeom(c.n_layer, c.n_embd, c.n_head, c.n_query_groups, c.head_size, c.intermediate_size,
                               lm.out_features, kv.k.size(-2), lm.group, lm.fmt, self.cos.size(0),
                               int(n_cu or ops.num_cus()), float(blocks[0].norm_1.eps), float(c.head_size ** -0.5))
        lib = engine_library()
        if lib.lga_engine_check(ctypes.byref(self.geom)) != 0:
            raise NotImplementedError(f"DecodeEngine: {lib.lga_last_error_string().decode()}")
        table = (EngineLayer * c.n_layer)()
        self._keep = []
        for i, b in enumerate(blocks):
            a, m = b.attn, b.mlp
            for t in (b.norm_1.weight, b.norm_2.weight):
                if t.dtype != torch.bfloat16 or not t.is_contiguous():
                    raise NotImplementedError("DecodeEngine: norm weights must be contiguous bf16")
            k, v = a.kv_cache.k, a.kv_cache.v
            if k.dtype != torch.bfloat16:
                a.kv_cache.k, a.kv_cache.v = k.to(torch.bfloat16), v.to(torch.bfloat16)
                k, v = a.kv_cache.k, a.kv_cache.v
            table[i] = EngineLayer(a.attn.qweight.data_ptr(), a.attn.scales.data_ptr(), a.proj.qweight.data_ptr(),
                                   a.proj.scales.data_ptr(), m.fc_1.qweight.data_ptr(), m.fc_1.scales.data_ptr(),
                                   m.fc_2.qweight.data_ptr(), m.fc_2.scales.data_ptr(), m.proj.qweight.data_ptr(),
                                   m.proj.scales.data_ptr(), b.norm_1.weight.data_ptr(), b.norm_2.weight.data_ptr(),
                                   k.data_ptr(), v.data_ptr())
        raw = bytes(table)
        self.layers = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
        nbytes = lib.lga_engine_scratch_bytes(ctypes.byref(self.geom))
        self.scratch = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
        self.logits = torch.empty(lm.out_features, dtype=torch.bfloat16, device=dev)
        x0 = lib.lga_engine_x0(ctypes.byref(self.geom), ctypes.c_void_p(self.scratch.data_ptr()))
        off = x0 - self.scratch.data_ptr()
        self.x0 = self.scratch[off:off + 2 * c.n_embd].view(torch.bfloat16)
        self._lm = lm
        self._ln_f = model.transformer.ln_f.weight
        self._wte = model.transformer.wte.weight

    @staticmethod
    def supported(model) -> Tuple[bool, str]:
        why = _why_not(model)
        if why is None:
            c, lm = model.config, model.lm_head
            kv = model.transformer.h[0].attn.kv_cache
            g = EngineGeom(c.n_layer, c.n_embd, c.n_head, c.n_query_groups, c.head_size, c.intermediate_size,
                           lm.out_features, kv.k.size(-2), lm.group, lm.fmt, model.cos.size(0), ops.num_cus(),
                           1e-5, 1.0)
            lib = engine_library()
            if lib.lga_engine_check(ctypes.byref(g)) != 0:
                why = lib.lga_last_error_string().decode()
        return why is None, why or ""

    def set_embedding(self, emb: torch.Tensor) -> None:
        """The step's input: transformer.wte(token) (n_embd bf16); each step leaves the next one's here itself."""
        self.x0.copy_(emb.reshape(-1))

    def step(self, pos: torch.Tensor, token: Optional[torch.Tensor] = None, out_idx: Optional[torch.Tensor] = None,
             op_limit: int = 0) -> None:
        """One decode step at input_pos ``pos`` (int64, 1 element on the device, advanced by the step); the new
        token lands in ``token`` (int32) / ``out_idx`` (int64) and the next step's embedding in ``x0``."""
        if pos.dtype != torch.int64 or not pos.is_cuda:
            raise TypeError("pos must be an int64 GPU tensor")
        lm = self._lm
        _check(engine_library().lga_decode_engine(
            ctypes.byref(self.geom), self.layers.data_ptr(), lm.qweight.data_ptr(), lm.scales.data_ptr(),
            self._ln_f.data_ptr(), self._wte.data_ptr(), self.cos.data_ptr(), self.sin.data_ptr(), pos.data_ptr(),
            None if token is None else token.data_ptr(), None if out_idx is None else out_idx.data_ptr(),
            self.logits.data_ptr(), self.scratch.data_ptr(), int(op_limit), ops._stream()))

    def errors(self) -> int:
        """Non-zero after a launch that gave up waiting (syncs)."""
        e = ctypes.c_uint(0)
        _check(engine_library().lga_engine_error(ctypes.byref(self.geom), ctypes.c_void_p(self.scratch.data_ptr()),
                                                       ctypes.byref(e)))
        return int(e.value)

    def reset(self) -> None:
        """Zero the counters / epoch / error words (after an error, or after op_limit test launches)."""
        _check(engine_library().lga_engine_reset(ctypes.byref(self.geom),
                                                       ctypes.c_void_p(self.scratch.data_ptr()), ops._stream()))

    def check(self) -> None:
        e = self.errors()
        if e:
            self.reset()
            raise EngineTimeout(f"decode engine launch gave up waiting (error bits {e:#x}); state reset")

    # the per-layer activations in the scratch (tests): plain bf16; the step input x0 and x[l] = block l-1's output
    def buffer(self, name: str, layer: int) -> torch.Tensor:
        c = self.model.config
        if name == "x" and layer == 0:
            return self.x0
        lay = (ctypes.c_longlong * 8)()
        _check(engine_library().lga_engine_layout(ctypes.byref(self.geom), lay))
        o_x0, o_act, act_len, a_qkv, a_y, a_xp, a_g, a_x = list(lay)
        sizes = {"qkv": ((c.n_head + 2 * c.n_query_groups) * c.head_size, a_qkv), "y": (c.n_embd, a_y),
                 "xp": (c.n_embd, a_xp), "g": (c.intermediate_size, a_g), "x": (c.n_embd, a_x)}
        n, off = sizes[name]
        blk = layer - 1 if name == "x" else layer
        base = o_act + act_len * blk + 2 * off
        return self.scratch[base:base + 2 * n].view(torch.bfloat16)
