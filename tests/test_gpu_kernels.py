"""Per-kernel parity on the MI355X: every HIP op through the C-ABI against the CPU oracle.

Integer / byte work (quantizer packing, KV append, argmax) must be bit-exact; fp kernels are checked against an
fp64/fp32 reference of the same op on the same bf16 inputs with the tolerance written in each test.
"""

import math

import numpy as np
import pytest
import torch

from oracle import model as om
from oracle import quant, synth

pytestmark = pytest.mark.gpu

DEV = "cuda"


def bf16_np(x: np.ndarray) -> np.ndarray:
    return quant.bf16_bits_to_f32(quant.f32_to_bf16_bits(x))


def to_dev_bf16(x: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(DEV).to(torch.bfloat16)


@pytest.fixture(scope="module")
def ops():
    from lit_gpt import ops as _ops

    _ops.load_library()
    return _ops


_CACHE = {}


def _weights(N, K, name, std=0.02):
    key = ("w", N, K, name)
    if key not in _CACHE:
        seed = abs(hash((N, K, name))) % (2 ** 31)
        _CACHE[key] = (np.random.default_rng(seed).standard_normal((N, K), dtype=np.float32) * std)
    return _CACHE[key]


# ------------------------------------------------------------------------------------------------ quantizer
@pytest.mark.parametrize("fmt,group", [(0, 128), (0, 64), (0, 32), (1, 64), (3, 64)])
@pytest.mark.parametrize("in_bf16", [False, True])
def test_quantizer_bit_exact(ops, fmt, group, in_bf16):
    w = _weights(96, 512, f"qz{fmt}{group}")
    w[3, :group] = 0.0  # an all-zero group (scale 0)
    w[5, 7] = 0.5  # an outlier
    if fmt == 3:  # every fp4 pivot exactly, just below and just above (relative to the block absmax 0.5)
        piv = quant.FP4_PIVOTS.astype(np.float32) * np.float32(0.5)
        edge = np.concatenate([piv, np.nextafter(piv, np.float32(0)), np.nextafter(piv, np.float32(1))])
        w[5, 8:8 + edge.size] = edge
        w[5, 32:32 + edge.size] = -edge
    if in_bf16:
        w = bf16_np(w)
    wt = torch.from_numpy(w).to(DEV)
    if in_bf16:
        wt = wt.to(torch.bfloat16)
    qw, sc = ops.quantize(wt, fmt, group)
    if fmt == 0:
        p_ref, s_ref = quant.quantize_q4g(w, group)
        np.testing.assert_array_equal(sc.view(torch.int16).cpu().numpy().view(np.uint16), s_ref)
    else:
        p_ref, s_ref = quant.quantize_fmt(w, fmt, group)
        np.testing.assert_array_equal(sc.cpu().numpy(), s_ref)
    np.testing.assert_array_equal(qw.cpu().numpy(), p_ref)


# ------------------------------------------------------------------------------------------------ GEMV
@pytest.mark.parametrize("n", [1, 255, 256, 4096 * 64 // 64 * 3 + 17, 11008 * 4096 // 64])
def test_nf4_double_quant_bit_exact(ops, n):
    """lga_nf4_double_quant == oracle/quant.py double_quant_absmax (bitsandbytes compress_statistics restated):
    every dequantized statistic bit-identical, the offset too."""
    from lit_gpt.quantize import bnb_dynamic_map

    rng = np.random.default_rng(n)
    a = (np.abs(rng.standard_normal(n)) * 0.05 + 0.01).astype(np.float32)
    if n >= 256:
        a[:256] = np.float32(0.03)  # a block whose centred values are all equal (absmax2 can be tiny / zero)
    dev = torch.from_numpy(a.copy()).to(DEV)
    off = ops.nf4_double_quant(dev, bnb_dynamic_map(DEV))
    q, amax2, offset, ref = quant.double_quant_absmax(a)
    assert float(off.item()) == float(offset)
    np.testing.assert_array_equal(dev.cpu().numpy(), ref)


def _ref_linear(x, wdeq, bias=None):
    y = x.astype(np.float64) @ wdeq.astype(np.float64).T
    return y if bias is None else y + bias


def _deq(ops, w, fmt, group):
    key = ("d", id(w), fmt, group)
    if key not in _CACHE:
        _CACHE[key] = quant.dequantize_fmt(*quant.quantize_fmt(w, fmt, group), fmt, group)
    return _CACHE[key]


@pytest.mark.parametrize("fmt,group", [(0, 128), (1, 64), (0, 32), (3, 64)])
@pytest.mark.parametrize("N,K", [(12288, 4096), (4096, 11008), (1000, 256), (77, 1376), (640, 4096)])
@pytest.mark.parametrize("variant", [-1, 0, 3, 4, 38])  # 4 / 38: the streaming form (2 / 3 workgroups per CU)
def test_gemv_matches_reference(ops, fmt, group, N, K, variant):
    if K % group:
        pytest.skip("group does not divide K")
    w = _weights(N, K, f"gv{N}x{K}")
    x = bf16_np(synth.normal((K,), f"x{K}", 5, 1.0))
    wt = torch.from_numpy(w).to(DEV)
    qw, sc = ops.quantize(wt, fmt, group)
    y = ops.q4_gemv(to_dev_bf16(x), qw, sc, N, K, group, fmt, variant=variant).float().cpu().numpy()
    ref = _ref_linear(x, _deq(ops, w, fmt, group))
    # bf16 output rounding (2^-8 relative) + fp32 accumulation differences
    tol = np.abs(ref) * 2 ** -7 + 1e-3 * np.sqrt(K / 4096) * 0.02 * np.abs(x).mean() * 4
    assert np.all(np.abs(y - ref) <= tol), float(np.max(np.abs(y - ref) - tol))


@pytest.mark.parametrize("fmt,group", [(0, 128), (1, 64), (3, 64)])
def test_gemv_fused_norm_residual_bias(ops, fmt, group):
    N, K = 1536, 1024
    w = _weights(N, K, "gvf")
    x = bf16_np(synth.normal((K,), "xf", 5, 2.0))
    nw = bf16_np(1.0 + synth.normal((K,), "nw", 5, 0.2))
    res = bf16_np(synth.normal((N,), "res", 5, 1.0))
    bias = bf16_np(synth.normal((N,), "bias", 5, 0.1))
    qw, sc = ops.quantize(torch.from_numpy(w).to(DEV), fmt, group)
    y = ops.q4_gemv(to_dev_bf16(x), qw, sc, N, K, group, fmt, bias=to_dev_bf16(bias), residual=to_dev_bf16(res),
                    norm_weight=to_dev_bf16(nw), eps=1e-5).float().cpu().numpy()
    xn = om.rms_norm(torch.from_numpy(x).bfloat16(), torch.from_numpy(nw).bfloat16(), 1e-5).float().numpy()
    h = bf16_np((_ref_linear(xn, _deq(ops, w, fmt, group)) + bias).astype(np.float32))
    ref = h + res
    assert np.max(np.abs(y - ref) - np.abs(ref) * 2 ** -7 - np.abs(h) * 2 ** -7) <= 2e-3


@pytest.mark.parametrize("fmt,group", [(0, 128), (1, 64), (3, 64)])
@pytest.mark.parametrize("variant", [-1, 0, 1, 36])  # -1 picks the streaming form at this shape, 0 / 1 one-shot
def test_gemv_swiglu(ops, fmt, group, variant):
    N, K = 11008, 4096
    w1, w2 = _weights(N, K, "s1"), _weights(N, K, "s2")
    x = bf16_np(synth.normal((K,), "xs", 5, 1.0))
    nw = bf16_np(np.ones(K, np.float32))
    q1, s1 = ops.quantize(torch.from_numpy(w1).to(DEV), fmt, group)
    q2, s2 = ops.quantize(torch.from_numpy(w2).to(DEV), fmt, group)
    y = ops.q4_gemv_swiglu(to_dev_bf16(x), q1, s1, q2, s2, N, K, group, fmt, norm_weight=to_dev_bf16(nw),
                           variant=variant).float().cpu().numpy()
    xn = om.rms_norm(torch.from_numpy(x).bfloat16(), torch.from_numpy(nw).bfloat16(), 1e-5).float().numpy()
    a = _ref_linear(xn, _deq(ops, w1, fmt, group))
    b = _ref_linear(xn, _deq(ops, w2, fmt, group))
    ref = (a / (1 + np.exp(-a))) * b
    assert np.max(np.abs(y - ref) - np.abs(ref) * 2 ** -6) <= 1e-3


# ------------------------------------------------------------------------------------------------ GEMM (prefill)
@pytest.mark.parametrize("fmt,group", [(0, 128), (1, 64), (3, 64)])
@pytest.mark.parametrize("M,N,K", [(200, 768, 256), (2048, 1024, 4096), (5, 640, 1376), (130, 4096, 11008)])
def test_gemm_matches_reference(ops, fmt, group, M, N, K):
    if K % group:
        group = 32 if fmt == 0 else pytest.skip("nf4 block must divide K")
    w = _weights(N, K, f"gm{N}x{K}")
    x = bf16_np(synth.normal((M, K), f"gx{M}x{K}", 5, 1.0))
    qw, sc = ops.quantize(torch.from_numpy(w).to(DEV), fmt, group)
    res = bf16_np(synth.normal((M, N), "gres", 5, 1.0))
    y = ops.q4_gemm(to_dev_bf16(x), qw, sc, N, K, group, fmt, residual=to_dev_bf16(res)).float().cpu().numpy()
    # the MFMA is fed bf16(value * scale) — the reference's dequantize-to-bf16-then-GEMM rounding
    wd = bf16_np(_deq(ops, w, fmt, group))
    h = _ref_linear(x, wd)
    ref = bf16_np(h.astype(np.float32)) + res
    err = np.abs(y - ref) - (np.abs(ref) + np.abs(h)) * 2 ** -7
    assert np.max(err) <= 2e-3, float(np.max(err))


@pytest.mark.parametrize("fmt,group", [(0, 128), (1, 64), (0, 32), (3, 64)])
@pytest.mark.parametrize("M,N,K", [(512, 768, 256), (600, 1024, 4096), (2048, 640, 1376), (517, 4096, 11008)])
def test_dequantize_then_bf16_gemm_is_q4_gemm(ops, fmt, group, M, N, K):
    """lga_q4_dequantize == the oracle's bf16(dequantize) bit for bit; gemm.hip's bf16 GEMM over it == lga_q4_gemm
    bit for bit (the same bf16 B tiles, the same MFMA order); QuantLinear's prefill path (the fused-dequant GEMM,
    or gemm.hip for group 32) within bf16 rounding of the fp64 product."""
    if K % group:
        group = 32
    w = _weights(N, K, f"dq{N}x{K}")
    qw, sc = ops.quantize(torch.from_numpy(w).to(DEV), fmt, group)
    wd = ops.q4_dequantize(qw, sc, N, K, group, fmt)
    np.testing.assert_array_equal(wd.float().cpu().numpy(), bf16_np(_deq(ops, w, fmt, group)))
    xn = bf16_np(synth.normal((M, K), f"dqx{M}x{K}", 5, 1.0))
    resn = bf16_np(synth.normal((M, N), "dqres", 5, 1.0))
    x, res = to_dev_bf16(xn), to_dev_bf16(resn)
    ref = ops.q4_gemm(x, qw, sc, N, K, group, fmt, residual=res)
    assert torch.equal(ops.bf16_gemm(x, wd, residual=res), ref)
    from lit_gpt.quantize import QuantLinear

    lin = QuantLinear(K, N, fmt, group, device=DEV)
    lin.qweight.copy_(qw)
    lin.scales.copy_(sc)
    y = lin(x, residual=res).float().cpu().numpy()  # the product's prefill GEMM: vs the fp64 product
    h = _ref_linear(xn, bf16_np(_deq(ops, w, fmt, group)))
    exp = bf16_np(h.astype(np.float32)) + resn
    assert np.max(np.abs(y - exp) - (np.abs(exp) + np.abs(h)) * 2 ** -7) <= 2e-3


# ------------------------------------------------------------------------------------------------ bf16 weights
# BASELINE config 2: unquantized nn.Linear in bf16-true. Reference: fp64 product of the same bf16 x and W.
@pytest.mark.parametrize("N,K", [(12288, 4096), (4096, 11008), (32000, 4096), (1000, 256), (77, 1376), (40, 8),
                                 (640, 8192), (300, 28672)])
def test_bf16_gemv_matches_reference(ops, N, K):
    w = bf16_np(_weights(N, K, f"bgv{N}x{K}"))
    x = bf16_np(synth.normal((K,), f"bx{K}", 5, 1.0))
    y = ops.bf16_gemv(to_dev_bf16(x), to_dev_bf16(w)).float().cpu().numpy()
    ref = _ref_linear(x, w)
    # bf16 output rounding (2^-8 relative) + fp32 accumulation order
    tol = np.abs(ref) * 2 ** -7 + 1e-3 * np.sqrt(K / 4096) * 0.02 * np.abs(x).mean() * 4
    assert np.all(np.abs(y - ref) <= tol), float(np.max(np.abs(y - ref) - tol))


@pytest.mark.parametrize("K", [1024, 11008])
def test_bf16_gemv_fused_norm_residual_bias(ops, K):
    N = 1536
    w = bf16_np(_weights(N, K, "bgvf"))
    x = bf16_np(synth.normal((K,), "bxf", 5, 2.0))
    nw = bf16_np(1.0 + synth.normal((K,), "bnw", 5, 0.2))
    res = bf16_np(synth.normal((N,), "bres", 5, 1.0))
    bias = bf16_np(synth.normal((N,), "bbias", 5, 0.1))
    y = ops.bf16_gemv(to_dev_bf16(x), to_dev_bf16(w), bias=to_dev_bf16(bias), residual=to_dev_bf16(res),
                      norm_weight=to_dev_bf16(nw), eps=1e-5).float().cpu().numpy()
    xn = om.rms_norm(torch.from_numpy(x).bfloat16(), torch.from_numpy(nw).bfloat16(), 1e-5).float().numpy()
    h = bf16_np((_ref_linear(xn, w) + bias).astype(np.float32))
    ref = h + res
    assert np.max(np.abs(y - ref) - np.abs(ref) * 2 ** -7 - np.abs(h) * 2 ** -7) <= 2e-3


@pytest.mark.parametrize("N,K", [(11008, 4096), (333, 8192)])
def test_bf16_gemv_swiglu(ops, N, K):
    w1, w2 = bf16_np(_weights(N, K, "bs1")), bf16_np(_weights(N, K, "bs2"))
    x = bf16_np(synth.normal((K,), "bxs", 5, 1.0))
    nw = bf16_np(1.0 + synth.normal((K,), "bnws", 5, 0.1))
    y = ops.bf16_gemv_swiglu(to_dev_bf16(x), to_dev_bf16(w1), to_dev_bf16(w2), norm_weight=to_dev_bf16(nw)
                             ).float().cpu().numpy()
    xn = om.rms_norm(torch.from_numpy(x).bfloat16(), torch.from_numpy(nw).bfloat16(), 1e-5).float().numpy()
    a, b = _ref_linear(xn, w1), _ref_linear(xn, w2)
    ref = (a / (1 + np.exp(-a))) * b
    assert np.max(np.abs(y - ref) - np.abs(ref) * 2 ** -6) <= 1e-3


@pytest.mark.parametrize("M,N,K", [(200, 768, 256), (2048, 1024, 4096), (5, 640, 1376), (130, 4096, 11008),
                                   (64, 96, 32), (300, 1000, 1376), (2048, 12288, 4096)])
@pytest.mark.parametrize("impl", ["mfma", "fused"])
def test_bf16_gemm_matches_reference(ops, M, N, K, impl):
    """Both bf16 GEMMs (gemm.hip's 128 x 128 MFMA tiles; gemm_q4f.hip's tiles with the weight DMA'd as stored, the
    unquantized model's prefill path) vs an fp64 product of the same bf16 operands, bias in the product, residual
    added after the bf16 rounding (Block's `proj(y) + h`)."""
    if impl == "fused" and not ops.q4f_fits(M, N, K, 64, 2):
        pytest.skip("shape outside the fused kernel (K % 64)")
    w = bf16_np(_weights(N, K, f"bgm{N}x{K}"))
    x = bf16_np(synth.normal((M, K), f"bgx{M}x{K}", 5, 1.0))
    res = bf16_np(synth.normal((M, N), "bgres", 5, 1.0))
    bias = bf16_np(synth.normal((N,), "bgbias", 5, 0.1))
    args = (to_dev_bf16(x), to_dev_bf16(w))
    kw = dict(bias=to_dev_bf16(bias), residual=to_dev_bf16(res))
    if impl == "fused":
        y = ops.q4_gemm_fused(args[0], args[1], None, N, K, 64, 2, **kw).float().cpu().numpy()
    else:
        y = ops.bf16_gemm(*args, **kw).float().cpu().numpy()
    h = _ref_linear(x, w) + bias
    ref = bf16_np(h.astype(np.float32)) + res
    err = np.abs(y - ref) - (np.abs(ref) + np.abs(h)) * 2 ** -7
    assert np.max(err) <= 2e-3, float(np.max(err))


def test_bf16_ops_reject_bad_arguments(ops):
    w = torch.zeros(16, 12, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(RuntimeError, match="multiple of 8"):
        ops.bf16_gemv(torch.zeros(12, dtype=torch.bfloat16, device=DEV), w)
    with pytest.raises(TypeError):
        ops.bf16_gemv(torch.zeros(16, device=DEV), torch.zeros(4, 16, device=DEV))
    with pytest.raises(RuntimeError, match="multiple of 32"):
        ops.bf16_gemm(torch.zeros(2, 16, dtype=torch.bfloat16, device=DEV),
                      torch.zeros(4, 16, dtype=torch.bfloat16, device=DEV))


# ------------------------------------------------------------------------------------------------ row ops
def test_rmsnorm_matches_oracle(ops, golden):
    g = golden("g3_ops.npz")
    x = torch.from_numpy(g["rms_x"]).bfloat16()
    w = torch.from_numpy(g["rms_w"]).bfloat16()
    y = ops.rmsnorm(x.to(DEV), w.to(DEV), 1e-5).float().cpu()
    ref = om.rms_norm(x, w, 1e-5).float()
    # one bf16 ulp: the fp32 sum of squares is reduced in a different order than torch's CPU mean
    assert torch.all((y - ref).abs() <= ref.abs() * 2 ** -7 + 1e-6)
    assert (y == ref).float().mean() > 0.97


@pytest.mark.parametrize("rows,n", [(2048, 4096), (3, 8192), (5, 1000), (7, 4100), (2, 11008)])
def test_rmsnorm_vector_and_scalar_forms(ops, rows, n):
    """16-B form (n % 8 == 0, n <= 8192) and the scalar fallback (n = 4100, and 11008 > 8192) vs the oracle's
    RMSNorm, one bf16 ulp (fp32 sums of squares in different orders)."""
    x = torch.from_numpy(synth.normal((rows, n), f"rmx{n}", 5, 2.0)).bfloat16()
    w = torch.from_numpy(1.0 + synth.normal((n,), f"rmw{n}", 5, 0.2)).bfloat16()
    y = ops.rmsnorm(x.to(DEV), w.to(DEV), 1e-5).float().cpu()
    ref = om.rms_norm(x, w, 1e-5).float()
    assert torch.all((y - ref).abs() <= ref.abs() * 2 ** -7 + 1e-6)
    assert (y == ref).float().mean() > 0.97


@pytest.mark.parametrize("H,G,hs,n_elem", [(32, 32, 128, 128), (8, 2, 128, 128), (4, 1, 64, 64), (12, 12, 64, 16),
                                           (4, 2, 80, 20)])  # the last: scalar kernel (half not a multiple of 8)
def test_rope_kv_append_bit_exact(ops, H, G, hs, n_elem):
    T, S = 7, 40
    qkv = bf16_np(synth.normal((T, (H + 2 * G) * hs), "qkv", 5, 1.0))
    cos, sin = om.build_rope_cache(S, n_elem, 10000)
    pos = torch.tensor([3, 4, 5, 6, 7, 8, 30])
    kc = torch.zeros(G, S, hs, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    q = ops.rope_kv_append(to_dev_bf16(qkv), kc, vc, pos.to(DEV), pos.to(DEV), cos.to(DEV), sin.to(DEV), H, G, hs,
                           n_elem).float().cpu()
    qpk = H // G
    t = torch.from_numpy(qkv).bfloat16().view(T, G, qpk + 2, hs)
    c, s = cos[pos], sin[pos]
    rq = t[:, :, :qpk].reshape(T, H, hs).transpose(0, 1)
    rk = t[:, :, qpk].transpose(0, 1)
    rq = torch.cat((om.apply_rope(rq[..., :n_elem], c, s), rq[..., n_elem:]), -1).transpose(0, 1)
    rk = torch.cat((om.apply_rope(rk[..., :n_elem], c, s), rk[..., n_elem:]), -1)
    assert torch.equal(q, rq.float())
    kref = torch.zeros(G, S, hs, dtype=torch.bfloat16)
    vref = torch.zeros_like(kref)
    kref[:, pos] = rk
    vref[:, pos] = t[:, :, qpk + 1].transpose(0, 1)
    assert torch.equal(kc.cpu(), kref) and torch.equal(vc.cpu(), vref)


@pytest.mark.parametrize("H,G,hs", [(32, 32, 128), (64, 8, 128), (8, 1, 128), (4, 2, 64)])
@pytest.mark.parametrize("T,positions", [(1, [0]), (1, [2047]), (1, [2302]), (5, [100, 101, 102, 103, 104]),
                                          (3, [0, 1, 2])])
@pytest.mark.parametrize("splits", [1, 8, 36, 256])
def test_attention_matches_reference(ops, H, G, hs, T, positions, splits):
    S = 2304
    q = bf16_np(synth.normal((T, H, hs), "aq", 5, 1.0))
    k = bf16_np(synth.normal((G, S, hs), "ak", 5, 1.0))
    v = bf16_np(synth.normal((G, S, hs), "av", 5, 1.0))
    pos = torch.tensor(positions, dtype=torch.int64)
    scale = 1.0 / math.sqrt(hs)
    y = ops.attention(to_dev_bf16(q), to_dev_bf16(k), to_dev_bf16(v), pos.to(DEV), H, G, hs, scale,
                      n_splits=splits).float().cpu().numpy().reshape(T, H, hs)
    qpk = H // G
    ref = np.zeros((T, H, hs))
    for t, p in enumerate(positions):
        for h in range(H):
            kk, vv = k[h // qpk, : p + 1].astype(np.float64), v[h // qpk, : p + 1].astype(np.float64)
            s = kk @ q[t, h].astype(np.float64) * scale
            e = np.exp(s - s.max())
            ref[t, h] = (e / e.sum()) @ vv
    assert np.max(np.abs(y - ref) - np.abs(ref) * 2 ** -7) <= 1e-4


@pytest.mark.parametrize("H,G,hs", [(8, 8, 128), (8, 2, 128), (4, 1, 64), (6, 3, 64)])
@pytest.mark.parametrize("T,start", [(16, 0), (100, 0), (300, 0), (77, 500), (64, 1), (1100, 0), (640, 37)])
def test_prefill_flash_attention_matches_reference(ops, H, G, hs, T, start):
    """T >= 16 takes the MFMA flash-attention kernel: query t attends keys 0..start+t of the cache (keys beyond
    the query block and past max_seq masked), fp64 softmax reference; bf16 P/V products -> 2^-7 relative."""
    S = start + T + 40
    q = bf16_np(synth.normal((T, H, hs), "pq", 9, 1.0))
    k = bf16_np(synth.normal((G, S, hs), "pk", 9, 1.0))
    v = bf16_np(synth.normal((G, S, hs), "pv", 9, 1.0))
    positions = list(range(start, start + T))
    pos = torch.tensor(positions, dtype=torch.int64)
    scale = 1.0 / math.sqrt(hs)
    y = ops.attention(to_dev_bf16(q), to_dev_bf16(k), to_dev_bf16(v), pos.to(DEV), H, G, hs, scale,
                      n_splits=1).float().cpu().numpy().reshape(T, H, hs)
    qpk = H // G
    ref = np.zeros((T, H, hs))
    for t, p in enumerate(positions):
        for h in range(H):
            kk, vv = k[h // qpk, : p + 1].astype(np.float64), v[h // qpk, : p + 1].astype(np.float64)
            s = kk @ q[t, h].astype(np.float64) * scale
            e = np.exp(s - s.max())
            ref[t, h] = (e / e.sum()) @ vv
    # P enters the PV product as bf16 (as SDPA's bf16 math does): ~2^-8 relative per term
    err = np.abs(y - ref) - np.abs(ref) * 2 ** -6
    assert np.max(err) <= 5e-3, float(np.max(err))


@pytest.mark.parametrize("S,T,start", [(100, 100, 0), (150, 40, 110), (77, 77, 0), (200, 16, 184)])
def test_prefill_flash_attention_partial_last_tile_stays_in_cache(ops, S, T, start):
    """max_seq % 64 != 0 and the prompt ends in the last partial key tile, with the K / V caches views at the start
    of a larger NaN-filled allocation: the tile loads past max_seq (and the one-tile-ahead prefetch) must read
    zeros through the buffer range check, never the bytes after the last group's cache (a NaN there times P = 0
    poisons the output). Finite and equal to the fp64 reference."""
    H, G, hs = 8, 2, 128
    q = bf16_np(synth.normal((T, H, hs), "tq", 11, 1.0))
    k = bf16_np(synth.normal((G, S, hs), "tk", 11, 1.0))
    v = bf16_np(synth.normal((G, S, hs), "tv", 11, 1.0))
    n = G * S * hs
    bufs = []
    for a in (k, v):  # NaN rows right after the last group's cache
        b = torch.full((n + 256 * hs,), float("nan"), dtype=torch.bfloat16, device=DEV)
        view = b[:n].view(G, S, hs)
        view.copy_(to_dev_bf16(a))
        bufs.append((b, view))
    positions = list(range(start, start + T))
    pos = torch.tensor(positions, dtype=torch.int64)
    scale = 1.0 / math.sqrt(hs)
    y = ops.attention(to_dev_bf16(q), bufs[0][1], bufs[1][1], pos.to(DEV), H, G, hs, scale,
                      n_splits=1).float().cpu().numpy().reshape(T, H, hs)
    assert np.all(np.isfinite(y))
    qpk = H // G
    ref = np.zeros((T, H, hs))
    for t, p in enumerate(positions):
        for h in range(H):
            kk, vv = k[h // qpk, : p + 1].astype(np.float64), v[h // qpk, : p + 1].astype(np.float64)
            s = kk @ q[t, h].astype(np.float64) * scale
            e = np.exp(s - s.max())
            ref[t, h] = (e / e.sum()) @ vv
    err = np.abs(y - ref) - np.abs(ref) * 2 ** -6
    assert np.max(err) <= 5e-3, float(np.max(err))


@pytest.mark.parametrize("H,G", [(32, 32), (64, 8), (8, 1), (16, 8)])
@pytest.mark.parametrize("p", [0, 1, 37, 2047, 2303])
@pytest.mark.parametrize("splits", [1, 7, 36])
def test_attention_decode_fused_matches_two_launch_path(ops, H, G, p, splits):
    """RoPE + KV-append + attention in one launch == lga_rope_kv_append then lga_attention: caches bit-exact,
    y within fp32 reordering (the new key is accumulated last), and both close to an fp64 softmax."""
    hs, S = 128, 2304
    qkv = to_dev_bf16(synth.normal((1, (H + 2 * G) * hs), "fq", 7, 1.0))
    k0 = to_dev_bf16(synth.normal((G, S, hs), "fk", 7, 1.0))
    v0 = to_dev_bf16(synth.normal((G, S, hs), "fv", 7, 1.0))
    cos, sin = om.build_rope_cache(S, hs, 10000)
    cos, sin = cos.to(DEV), sin.to(DEV)
    pos = torch.tensor([p], device=DEV)
    scale = 1.0 / math.sqrt(hs)
    ka, va = k0.clone(), v0.clone()
    q = ops.rope_kv_append(qkv, ka, va, pos, pos, cos, sin, H, G, hs, hs)
    ya = ops.attention(q, ka, va, pos, H, G, hs, scale, n_splits=splits).float()
    kb, vb = k0.clone(), v0.clone()
    yb = ops.attention_decode_fused(qkv, kb, vb, pos, pos, cos, sin, H, G, hs, hs, scale, n_splits=splits).float()
    assert torch.equal(ka, kb) and torch.equal(va, vb)
    assert torch.all((ya - yb).abs() <= ya.abs() * 2 ** -7 + 2e-3)
    # fp64 reference from the (bit-exact) cache contents
    qpk = H // G
    qd = q.double().cpu()
    kd, vd = ka[:, : p + 1].double().cpu(), va[:, : p + 1].double().cpu()
    ref = torch.empty(H, hs, dtype=torch.float64)
    for h in range(H):
        s = kd[h // qpk] @ qd[0, h] * scale
        ref[h] = torch.softmax(s, 0) @ vd[h // qpk]
    yb = yb.double().cpu().view(H, hs)
    assert torch.max((yb - ref).abs() - ref.abs() * 2 ** -7) <= 1e-4


@pytest.mark.parametrize("H,G", [(32, 32), (8, 1), (32, 8)])
@pytest.mark.parametrize("p", [1726, 1727, 2000, 2047, 2302, 2303])
@pytest.mark.parametrize("splits", [8, 16, 36])
def test_attention_decode_fixed_splits_ignore_rows_past_p(ops, H, G, p, splits):
    """Split ranges fixed by the cache length (csrc/attention.hip LGA_ATTN_FIXED: the first K/V batch leaves before
    input_pos is read, and may cover rows past p) with every cache row past p set to NaN: the output is finite and
    matches the fp64 softmax over keys 0..p; p = 1726 / 1727 sit on either side of the 3/4-of-the-cache switch to
    live-position ranges (S = 2304)."""
    hs, S = 128, 2304
    qkv = to_dev_bf16(synth.normal((1, (H + 2 * G) * hs), "nq", 8, 1.0))
    k0 = to_dev_bf16(synth.normal((G, S, hs), "nk", 8, 1.0))
    v0 = to_dev_bf16(synth.normal((G, S, hs), "nv", 8, 1.0))
    k0[:, p:] = float("nan")  # row p is appended by the launch itself
    v0[:, p:] = float("nan")
    cos, sin = om.build_rope_cache(S, hs, 10000)
    cos, sin = cos.to(DEV), sin.to(DEV)
    pos = torch.tensor([p], device=DEV)
    scale = 1.0 / math.sqrt(hs)
    y = ops.attention_decode_fused(qkv, k0, v0, pos, pos, cos, sin, H, G, hs, hs, scale, n_splits=splits)
    y = y.double().cpu().view(H, hs)
    assert torch.all(torch.isfinite(y))
    qpk = H // G
    kd, vd = k0[:, : p + 1].double().cpu(), v0[:, : p + 1].double().cpu()
    q = ops.rope_kv_append(qkv, k0.clone(), v0.clone(), pos, pos, cos, sin, H, G, hs, hs).double().cpu()
    ref = torch.empty(H, hs, dtype=torch.float64)
    for h in range(H):
        sc = kd[h // qpk] @ q[0, h] * scale
        ref[h] = torch.softmax(sc, 0) @ vd[h // qpk]
    assert torch.max((y - ref).abs() - ref.abs() * 2 ** -7) <= 1e-4


def test_attention_decode_fused_rejects_unsupported_geometry(ops):
    qkv = torch.zeros(1, 3 * 64 * 4, dtype=torch.bfloat16, device=DEV)
    kc = torch.zeros(4, 16, 64, dtype=torch.bfloat16, device=DEV)
    cos = torch.ones(16, 64, device=DEV)
    pos = torch.zeros(1, dtype=torch.int64, device=DEV)
    with pytest.raises(RuntimeError, match="head_size == rope_n_elem == 128"):
        ops.attention_decode_fused(qkv, kc, kc.clone(), pos, pos, cos, cos, 4, 4, 64, 64, 0.125)


@pytest.mark.parametrize("splits", [16, 8])
def test_attention_split_counters_rearm_across_launches(ops, splits):
    """The in-launch split merge re-arms its counters: repeated launches on one workspace stay correct (16 splits x 32
    groups: more workgroups than CUs; 8 x 32: Llama-2-7B's decode geometry, one workgroup per CU)."""
    H, G, hs, S = 32, 32, 128, 2304
    q = to_dev_bf16(synth.normal((1, H, hs), "rq", 5, 1.0))
    k = to_dev_bf16(synth.normal((G, S, hs), "rk", 5, 1.0))
    v = to_dev_bf16(synth.normal((G, S, hs), "rv", 5, 1.0))
    ws = ops.AttentionWorkspace(1, H, G, hs, splits, DEV)
    outs = []
    for p in (2047, 5, 2047, 0, 2047):
        pos = torch.tensor([p], device=DEV)
        outs.append(ops.attention(q, k, v, pos, H, G, hs, 0.1, n_splits=splits, workspace=ws).clone())
    assert torch.equal(outs[0], outs[2]) and torch.equal(outs[0], outs[4])
    assert int(ws.counters.abs().sum()) == 0
    ref0 = v[:, 0].reshape(-1)  # position 0: softmax over one key -> exactly v[0]
    assert torch.equal(outs[3].view(-1), ref0)


def test_argmax_known_answers_and_ties(ops, golden):
    g = golden("g3_ops.npz")
    logits = torch.from_numpy(g["sample_logits"]).float()
    assert ops.argmax(logits[0, -1].bfloat16().to(DEV)).item() == int(g["sample_t0"][0])
    tl = torch.from_numpy(g["sample_ties_logits"])[0, -1]
    assert ops.argmax(tl.bfloat16().to(DEV)).item() == int(g["sample_ties_t0"][0])
    big = torch.full((32000,), -3.0)
    big[[17, 31999, 20000]] = 5.0
    tok = torch.zeros(1, dtype=torch.int32, device=DEV)
    pos = torch.tensor([41], device=DEV)
    assert ops.argmax(big.bfloat16().to(DEV), token_out=tok, pos_inout=pos).item() == 17
    assert tok.item() == 17 and pos.item() == 42


@pytest.mark.parametrize("n", [1, 7, 8, 1001, 32000, 65549, 150001])
@pytest.mark.parametrize("offset", [0, 1])
def test_argmax_matches_torch_random(ops, n, offset):
    """Vector path (16-B aligned) and scalar path (odd offset), multi-pass vocabularies, ties, NaN."""
    g = torch.Generator().manual_seed(n + offset)
    x = (torch.randint(-50, 50, (n + offset,), generator=g).float() / 4).bfloat16()  # many exact ties
    view = x[offset:]
    dev = x.to(DEV)[offset:]
    assert ops.argmax(dev).item() == int(torch.argmax(view.float()))
    if n > 3:
        x2 = x.clone()
        x2[offset + n // 2] = float("nan")
        x2[offset + n - 1] = float("nan")
        assert ops.argmax(x2.to(DEV)[offset:]).item() == n // 2  # first NaN wins (torch.argmax)
    neg = torch.full((n,), float("-inf")).bfloat16()
    assert ops.argmax(neg.to(DEV)).item() == 0


@pytest.mark.parametrize("n,offset", [(32000, 0), (1001, 1), (7, 0)])
def test_argmax_embed_is_argmax_then_embedding(ops, n, offset):
    """lga_argmax_embed == lga_argmax followed by lga_embedding of the chosen token: same token, same token /
    position bookkeeping, the same embedding row bit for bit (ties, NaN, and a token past the table clamp as the
    embedding does)."""
    C = 4096
    V = max(n - 3, 1)  # the last logits index past the table: clamped to row V - 1 like lga_embedding
    table = to_dev_bf16(synth.normal((V, C), "aemb", 5, 1.0))
    g = torch.Generator().manual_seed(n)
    x = (torch.randint(-50, 50, (n + offset,), generator=g).float() / 4).bfloat16()
    cases = [x]
    if n > 3:
        x2 = x.clone()
        x2[offset + n // 3] = float("nan")
        cases.append(x2)
        x3 = x.clone()
        x3[offset + n - 1] = 100.0  # winner beyond the table's last row
        cases.append(x3)
    for xc in cases:
        lg = xc.to(DEV)[offset:]
        tok_a = torch.zeros(1, dtype=torch.int32, device=DEV)
        pos_a = torch.tensor([7], device=DEV)
        ia = ops.argmax(lg, token_out=tok_a, pos_inout=pos_a)
        emb_a = ops.embedding(tok_a, table).view(-1)
        tok_b = torch.zeros(1, dtype=torch.int32, device=DEV)
        pos_b = torch.tensor([7], device=DEV)
        emb_b = torch.empty(C, dtype=torch.bfloat16, device=DEV)
        ib = ops.argmax_embed(lg, table, emb_b, token_out=tok_b, pos_inout=pos_b)
        assert ia.item() == ib.item() == int(torch.argmax(xc[offset:].float()))
        assert tok_a.item() == tok_b.item() and pos_a.item() == pos_b.item() == 8
        assert torch.equal(emb_a, emb_b)


def test_embedding_and_add(ops):
    V, C = 500, 256
    table = bf16_np(synth.normal((V, C), "emb", 5, 1.0))
    idx = torch.tensor([3, 499, 0, 3], dtype=torch.int32)
    out = ops.embedding(idx.to(DEV), to_dev_bf16(table)).float().cpu().numpy()
    np.testing.assert_array_equal(out, table[idx.numpy()])
    a, b = to_dev_bf16(table[:4]), to_dev_bf16(table[4:8])
    assert torch.equal(ops.add(a, b), (a.float() + b.float()).bfloat16())


@pytest.mark.parametrize("n", [8, 4096, 2048 * 11008])
def test_vector_elementwise_equals_scalar(ops, n):
    """lga_add / lga_swiglu take 16-B vector kernels when n % 8 == 0: same bits as the scalar kernels (odd n)."""
    a = (torch.randn(n + 1, device=DEV) * 3).bfloat16()
    b = (torch.randn(n + 1, device=DEV) * 3).bfloat16()
    assert torch.equal(ops.add(a[:n], b[:n]), (a[:n].float() + b[:n].float()).bfloat16())
    vec = ops.swiglu(a[:n], b[:n])
    sca = ops.swiglu(a[: n + 1], b[: n + 1])  # n + 1 is odd: the scalar kernel
    assert torch.equal(vec, sca[:n])


def test_errors_are_raised(ops):
    x = torch.zeros(100, dtype=torch.bfloat16, device=DEV)
    qw = torch.zeros(10, 50, dtype=torch.uint8, device=DEV)
    sc = torch.zeros(10, 1, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(RuntimeError, match="multiple of 32"):
        ops.q4_gemv(x, qw, sc, 10, 100, 100, 0)
    with pytest.raises(RuntimeError, match="GPU tensor"):
        ops.rmsnorm(torch.zeros(4, 8, dtype=torch.bfloat16), torch.ones(8, dtype=torch.bfloat16), 1e-5)


# ------------------------------------------------------------------------------------------------ sparse MoE
def test_moe_route_matches_cpu_topk_on_ties(ops):
    """lga_moe_route == torch.topk on the CPU (the reference's tie order, model.py:737) + fp32 softmax cast to
    bf16 (model.py:738): ids bit-exact; probs bit-exact except a 1-ulp fp32 exp difference may move a bf16
    rounding (checked: <= 1 bf16 ulp)."""
    g = torch.Generator().manual_seed(3)
    rows = []
    for E in (8, 4, 6):
        pools = [torch.tensor([0.0, 1.0, 2.0]), torch.tensor([0.0, -0.0, 1.0, 1.5]), torch.arange(5.0), None]
        for pool in pools:
            if pool is None:
                v = torch.randn(400, E, generator=g)
            else:
                v = pool[torch.randint(0, pool.numel(), (400, E), generator=g)]
            rows.append((E, v.bfloat16()))
    for E, logits in rows:
        for k in (1, 2, 3):
            ids, probs = ops.moe_route(logits.to(DEV), k)
            pv, pi = torch.topk(logits, k)
            ref_p = pv.softmax(dim=1, dtype=torch.float).to(torch.bfloat16)
            assert torch.equal(ids.cpu().long(), pi), (E, k)
            d = (probs.cpu().view(torch.int16).int() - ref_p.view(torch.int16).int()).abs()
            assert int(d.max()) <= 1, (E, k)


@pytest.mark.parametrize("fmt,group", [(0, 128), (1, 64), (3, 64), (0, 32)])
@pytest.mark.parametrize("K", [4096, 1024, 6144, 2080])
def test_moe_gate_route_matches_gemv_then_route(ops, fmt, group, K):
    """lga_moe_gate_route (one launch) == lga_q4_gemv of the gate rows + lga_moe_route, bit for bit: with and without
    the fused RMSNorm, 4 / 6 / 8 experts, k = 1 / 2, and gate rows duplicated so the router logits tie."""
    if K % group:
        pytest.skip("K must be a multiple of the group")
    g = torch.Generator().manual_seed(K + fmt)
    for E in (8, 6, 4):
        w = torch.randn(E, K, generator=g) * 0.02
        if E == 8:
            w[5] = w[2]  # tied logits: the CPU torch.topk tie order decides
        qw, sc = ops.quantize(w.to(DEV), fmt, group)
        for norm in (False, True):
            x = torch.randn(K, generator=g).bfloat16().to(DEV)
            nw = (1.0 + 0.1 * torch.randn(K, generator=g)).bfloat16().to(DEV) if norm else None
            router = ops.q4_gemv(x, qw, sc, E, K, group, fmt, norm_weight=nw, eps=1e-5)
            for k in (1, 2):
                ids0, p0 = ops.moe_route(router.view(1, E), k)
                ids1, p1 = ops.moe_gate_route(x, qw, sc, E, K, group, fmt, k, norm_weight=nw, eps=1e-5)
                assert torch.equal(ids0, ids1), (E, norm, k, ids0, ids1)
                assert torch.equal(p0.view(torch.int16), p1.view(torch.int16)), (E, norm, k)


@pytest.mark.parametrize("fmt,group", [(0, 128), (1, 64), (3, 64), (0, 32)])
@pytest.mark.parametrize("N,K", [(4096, 14336), (512, 384), (1024, 2080), (768, 4096), (640, 6144), (512, 11008)])
def test_experts_pair_combine_matches_gemv_then_combine(ops, fmt, group, N, K):
    """lga_q4_gemv_experts_pair_combine (both slots' routed proj GEMVs, the second-arriving workgroup of each row block
    combining) == lga_q4_gemv_experts + lga_moe_combine (+ residual), bit for bit: both slot orders, every
    chunks-per-lane template, repeated launches (the counters re-arm) and a graph replay."""
    if K % group:
        pytest.skip("K must be a multiple of the group")
    assert ops.experts_pair_supported(N, K, group, fmt)
    g = torch.Generator().manual_seed(N + K + fmt + 7)
    E = 8
    qw, sc = [], []
    for e in range(E):
        q, s_ = ops.quantize((torch.randn(N, K, generator=g) * 0.02).to(DEV), fmt, group)
        qw.append(q)
        sc.append(s_)
    qw, sc = torch.stack(qw), torch.stack(sc)
    ws = ops.ExpertsPairWorkspace(N, DEV)
    for pair in ((1, 6), (6, 1), (0, 7), (3, 3)):
        ids = torch.tensor(pair, dtype=torch.int32, device=DEV)
        x = torch.randn(2, K, generator=g).bfloat16().to(DEV)
        probs = torch.softmax(torch.randn(2, generator=g), 0).bfloat16().to(DEV)
        res = (torch.randn(N, generator=g) * 2).bfloat16().to(DEV)
        eout = ops.q4_gemv_experts(x, qw, sc, ids, N, K, group, fmt)
        want = ops.moe_combine(eout.view(1, 2, N).contiguous(), probs.view(1, 2), ids.view(1, 2),
                               residual=res.view(1, N)).view(-1)
        got = ops.q4_gemv_experts_pair_combine(x, qw, sc, ids, probs, res, N, K, group, fmt, ws)
        assert torch.equal(got.view(torch.int16), want.view(torch.int16)), (pair, (got.float() - want.float()).abs().max())
    assert int(ws.counters.abs().sum()) == 0  # re-armed
    out = torch.empty(N, dtype=torch.bfloat16, device=DEV)
    ops.q4_gemv_experts_pair_combine(x, qw, sc, ids, probs, res, N, K, group, fmt, ws, out=out)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        ops.q4_gemv_experts_pair_combine(x, qw, sc, ids, probs, res, N, K, group, fmt, ws, out=out)
    for pair in ((5, 2), (2, 5)):
        ids.copy_(torch.tensor(pair, dtype=torch.int32))
        x.copy_(torch.randn(2, K, generator=g).bfloat16())
        graph.replay()
        torch.cuda.synchronize()
        eout = ops.q4_gemv_experts(x, qw, sc, ids, N, K, group, fmt)
        want = ops.moe_combine(eout.view(1, 2, N).contiguous(), probs.view(1, 2), ids.view(1, 2),
                               residual=res.view(1, N)).view(-1)
        assert torch.equal(out.view(torch.int16), want.view(torch.int16)), pair


def test_moe_gate_route_rejects_bad_shapes(ops):
    x = torch.zeros(8192, dtype=torch.bfloat16, device=DEV)
    qw, sc = ops.quantize(torch.zeros(8, 8192, device=DEV), 0, 128)
    with pytest.raises(RuntimeError, match="6144"):
        ops.moe_gate_route(x, qw, sc, 8, 8192, 128, 0, 2)
    with pytest.raises(RuntimeError, match="n_expert"):
        ops.moe_gate_route(x[:4096], qw, sc, 9, 4096, 128, 0, 2)


def test_moe_combine_matches_reference_loop(ops):
    """y[tok] += probs * expert_out in ascending expert order, bf16 arithmetic (model.py:739-742) + residual."""
    T, k, C = 9, 2, 4096
    g = torch.Generator().manual_seed(5)
    eout = torch.randn(T, k, C, generator=g).bfloat16()
    probs = torch.rand(T, k, generator=g).bfloat16()
    ids = torch.stack([torch.randperm(8, generator=g)[:k] for _ in range(T)]).int()
    res = torch.randn(T, C, generator=g).bfloat16()
    got = ops.moe_combine(eout.to(DEV), probs.to(DEV), ids.to(DEV), residual=res.to(DEV)).cpu()
    y = torch.zeros(T, C, dtype=torch.bfloat16)
    for e in range(8):
        tok, slot = torch.where(ids == e)
        y[tok] += probs[tok, slot, None] * eout[tok, slot]
    assert torch.equal(got, res + y)
    got_nores = ops.moe_combine(eout.to(DEV), probs.to(DEV), ids.to(DEV)).cpu()
    assert torch.equal(got_nores, y)


@pytest.mark.parametrize("fmt,group", [(0, 128), (1, 64), (3, 64)])
def test_routed_expert_gemvs_equal_per_expert_gemvs(ops, fmt, group):
    """Slot s of the routed GEMVs == the plain GEMV on expert ids[s]'s own weights (same kernel, bit-exact)."""
    E, N, K = 4, 1408, 512
    ws = [_weights(N, K, f"e{e}") for e in range(E)]
    qs = [ops.quantize(torch.from_numpy(w).to(DEV), fmt, group) for w in ws]
    qw = torch.stack([q for q, _ in qs])
    sc = torch.stack([s for _, s in qs])
    ws2 = [_weights(N, K, f"f{e}") for e in range(E)]
    qs2 = [ops.quantize(torch.from_numpy(w).to(DEV), fmt, group) for w in ws2]
    qw2 = torch.stack([q for q, _ in qs2])
    sc2 = torch.stack([s for _, s in qs2])
    ids = torch.tensor([3, 1], dtype=torch.int32, device=DEV)
    x = to_dev_bf16(synth.normal((K,), "xe", 5, 1.0))
    nw = to_dev_bf16(1.0 + 0.1 * synth.normal((K,), "nwe", 5, 1.0))
    act = ops.q4_gemv_swiglu_experts(x, qw, sc, qw2, sc2, ids, N, K, group, fmt, norm_weight=nw)
    for s, e in enumerate((3, 1)):
        ref = ops.q4_gemv_swiglu(x, qs[e][0], qs[e][1], qs2[e][0], qs2[e][1], N, K, group, fmt, norm_weight=nw)
        assert torch.equal(act[s], ref)
    # down projection: (K' = N) -> N' = K, each slot reading its own activation row
    wd = [_weights(K, N, f"d{e}") for e in range(E)]
    qd = [ops.quantize(torch.from_numpy(w).to(DEV), fmt, group) for w in wd]
    out = ops.q4_gemv_experts(act, torch.stack([q for q, _ in qd]), torch.stack([s for _, s in qd]), ids, K, N,
                              group, fmt)
    for s, e in enumerate((3, 1)):
        assert torch.equal(out[s], ops.q4_gemv(act[s].contiguous(), qd[e][0], qd[e][1], K, N, group, fmt))


@pytest.mark.parametrize("H,G,splits", [(8, 1, 16), (64, 8, 4), (16, 4, 16)])
def test_attention_decode_head_slices_agree(ops, H, G, splits, monkeypatch):
    """A query group's heads dealt to 1, 2, ... q_per_kv workgroups (LGA_ATTN_HSPLIT; by default when the groups
    are few): the same cache appends bit for bit, outputs within fp32 reordering of each other, and the split
    counters re-armed (two launches per setting on one workspace)."""
    hs, S, p = 128, 2304, 2303
    qkv = to_dev_bf16(synth.normal((1, (H + 2 * G) * hs), "hq", 3, 1.0))
    k0 = to_dev_bf16(synth.normal((G, S, hs), "hk", 3, 1.0))
    v0 = to_dev_bf16(synth.normal((G, S, hs), "hv", 3, 1.0))
    cos, sin = om.build_rope_cache(S, hs, 10000)
    cos, sin = cos.to(DEV), sin.to(DEV)
    pos = torch.tensor([p], device=DEV)
    scale = 1.0 / math.sqrt(hs)
    ws = ops.AttentionWorkspace(1, H, G, hs, splits, DEV)
    outs, caches = [], []
    for h in [x for x in (1, 2, 4, 8) if x <= H // G]:
        monkeypatch.setenv("LGA_ATTN_HSPLIT", str(h))
        for _ in range(2):
            kb, vb = k0.clone(), v0.clone()
            y = ops.attention_decode_fused(qkv, kb, vb, pos, pos, cos, sin, H, G, hs, hs, scale, n_splits=splits,
                                           workspace=ws).float()
        outs.append(y)
        caches.append((kb, vb))
    for y, (kb, vb) in zip(outs[1:], caches[1:]):
        assert torch.equal(kb, caches[0][0]) and torch.equal(vb, caches[0][1])
        assert torch.all((y - outs[0]).abs() <= outs[0].abs() * 2 ** -7 + 2e-3)


@pytest.mark.parametrize("mode,N,K", [("int4-g128", 32000, 4096), ("nf4", 32000, 4096), ("int4-g128", 50304, 2048),
                                      ("bnb.fp4", 1000, 256)])
@pytest.mark.parametrize("tie", [False, True])
def test_fused_greedy_head_bit_identical(ops, mode, N, K, tie):
    """lga_q4_gemv_argmax_embed (RMSNorm + lm_head GEMV + argmax + the next token's embedding row, one launch) ==
    lga_q4_gemv(norm) then lga_argmax_embed: logits, token, index, position and embedding row bit-identical; with
    ``tie`` the winning row is duplicated further down, so the lowest index must win (torch.argmax order). Several
    launches on one workspace (its arrival counters re-arm)."""
    from lit_gpt.quantize import QuantLinear

    g = torch.Generator().manual_seed(N + K)
    w = torch.randn(N, K, generator=g) * 0.02
    if tie:
        w[N // 3] = w[7] = torch.randn(K, generator=g) * 0.2  # two identical rows: equal logits
    lin = QuantLinear.from_float(w, None, mode, torch.device(DEV))
    nw = (1.0 + torch.randn(K, generator=g) * 0.1).bfloat16().to(DEV)
    table = torch.randn(N, 64, generator=g).bfloat16().to(DEV)
    work = ops.HeadWorkspace(N, K, DEV)
    for it in range(3):
        x = (torch.randn(K, generator=g) * 2).bfloat16().to(DEV)
        la = ops.q4_gemv(x, lin.qweight, lin.scales, N, K, lin.group, lin.fmt, norm_weight=nw)
        ia, ta, pa = (torch.zeros(1, dtype=torch.int64, device=DEV), torch.zeros(1, dtype=torch.int32, device=DEV),
                      torch.tensor([100 + it], device=DEV))
        ea = torch.empty(64, dtype=torch.bfloat16, device=DEV)
        ops.argmax_embed(la, table, ea, out_idx=ia, token_out=ta, pos_inout=pa)
        ib, tb, pb = torch.zeros_like(ia), torch.zeros_like(ta), torch.tensor([100 + it], device=DEV)
        eb = torch.empty_like(ea)
        lb = ops.q4_gemv_argmax_embed(x, lin, work, norm_weight=nw, table=table, emb_out=eb, out_idx=ib,
                                      token_out=tb, pos_inout=pb)
        assert torch.equal(la, lb) and int(ia) == int(ib) and int(ta) == int(tb) and int(pa) == int(pb) == 101 + it
        assert torch.equal(ea, eb)
        if tie and it == 0:
            assert int(ib) == 7 or float(la[int(ib)]) > float(la[7])
    assert int(work.buf[-(9 * 256) // 8:].abs().sum()) == 0  # counters re-armed

