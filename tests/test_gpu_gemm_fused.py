"""The prefill GEMM with the 4-bit dequantization fused in (lga_q4_gemm_fused / lga_q4_gemm_swiglu,
csrc/gemm_q4f.hip) against the oracle.

The reference's M > 1 Linear4bit path is dequantize_4bit to a bf16 weight, then the GEMM (bitsandbytes, reached
through BitsandbytesPrecision, reference generate/base.py:128-136): the kernel stages exactly those bf16 weights
(bf16(value(nibble) * scale), oracle/quant.py), so the product is compared with the fp64 product of the oracle's
dequantized weights, within bf16 rounding (tolerance in each test). LLaMAMLP's fc_1 / fc_2 / silu*mul
(reference model.py:712-716) is checked against bf16(bf16(silu(bf16(h1))) * bf16(h2)) of the fp64 products.
Shapes: ragged M (1, 17, 300, 513), N tails (136, 392: not multiples of the 128-column tile), K of one K-step
(64) up to Llama-2-7B's 11008, the 7B layer shapes at M = 2048 (fp32 GPU reference there).
"""

import numpy as np
import pytest
import torch

from oracle import quant, synth

pytestmark = pytest.mark.gpu
DEV = "cuda"


def bf16_np(x):
    return quant.bf16_bits_to_f32(quant.f32_to_bf16_bits(x))


def to_dev(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(DEV).to(torch.bfloat16)


@pytest.fixture(scope="module")
def ops():
    from lit_gpt import ops as _ops

    _ops.load_library()
    return _ops


def _w(N, K, tag, std=0.02):
    rng = np.random.default_rng(abs(hash((N, K, tag))) % (2 ** 31))
    return rng.standard_normal((N, K), dtype=np.float32) * std


def _quant(ops, w, fmt, group):
    qw, sc = ops.quantize(torch.from_numpy(w).to(DEV), fmt, group)
    p, s = quant.quantize_fmt(w, fmt, group)
    wd = quant.dequantize_fmt(p, s, fmt, group)
    return qw, sc, bf16_np(wd)


def _silu(v):
    return v / (1.0 + np.exp(-v))


def _swiglu_tol(a, b, g):
    """Bound on |g - g_ref| when the two products' bf16 roundings may each differ by one ulp (different fp32
    summation orders): |silu'| <= 1.1, so 2^-7 (1.1 |a| |b| + |silu(a)| |b|), + the final rounding + slack."""
    sa = a / (1.0 + (-a).exp()) if isinstance(a, torch.Tensor) else _silu(a)
    return 2 ** -7 * (1.1 * abs(a) * abs(b) + abs(sa) * abs(b)) + 2 ** -8 * abs(g) + 2e-3


@pytest.mark.parametrize("fmt,group", [(0, 128), (0, 64), (1, 64), (3, 64)])
@pytest.mark.parametrize("M,N,K", [(1, 128, 64), (17, 136, 256), (300, 392, 1024), (513, 256, 704)])
@pytest.mark.parametrize("epi", ["none", "residual", "bias+residual"])
def test_fused_gemm_matches_oracle(ops, fmt, group, M, N, K, epi):
    if K % group:
        pytest.skip("group must divide K")
    assert ops.q4f_fits(M, N, K, group, fmt)
    w = _w(N, K, "fg")
    qw, sc, wd = _quant(ops, w, fmt, group)
    x = bf16_np(synth.normal((M, K), f"fgx{M}x{K}", 5, 1.0))
    res = bf16_np(synth.normal((M, N), "fgres", 5, 1.0)) if "residual" in epi else None
    bias = bf16_np(synth.normal((N,), "fgb", 5, 0.1)) if "bias" in epi else None
    y = ops.q4_gemm_fused(to_dev(x), qw, sc, N, K, group, fmt, bias=None if bias is None else to_dev(bias),
                          residual=None if res is None else to_dev(res)).float().cpu().numpy()
    h = x.astype(np.float64) @ wd.astype(np.float64).T
    if bias is not None:
        h = h + bias
    ref = bf16_np(h.astype(np.float32))
    if res is not None:
        ref = ref + res
    err = np.abs(y - ref) - (np.abs(ref) + np.abs(h)) * 2 ** -7
    assert np.max(err) <= 2e-3, float(np.max(err))


@pytest.mark.parametrize("fmt,group", [(0, 128), (1, 64)])
@pytest.mark.parametrize("M,N,K", [(1, 64, 128), (40, 200, 512), (300, 392, 1024)])
def test_fused_swiglu_matches_oracle(ops, fmt, group, M, N, K):
    w1, w2 = _w(N, K, "s1"), _w(N, K, "s2")
    q1, s1, d1 = _quant(ops, w1, fmt, group)
    q2, s2, d2 = _quant(ops, w2, fmt, group)
    x = bf16_np(synth.normal((M, K), f"sx{M}x{K}", 5, 1.0))
    g = ops.q4_gemm_swiglu(to_dev(x), q1, s1, q2, s2, N, K, group, fmt).float().cpu().numpy()
    h1 = x.astype(np.float64) @ d1.astype(np.float64).T
    h2 = x.astype(np.float64) @ d2.astype(np.float64).T
    a = bf16_np(h1.astype(np.float32))
    ref = bf16_np(bf16_np(_silu(a.astype(np.float64)).astype(np.float32)) * bf16_np(h2.astype(np.float32)))
    err = np.abs(g - ref) - _swiglu_tol(a, bf16_np(h2.astype(np.float32)), ref)
    assert np.max(err) <= 0.0, float(np.max(err))


@pytest.mark.parametrize("M,N,K", [(2048, 4096, 4096), (2048, 4096, 11008), (257, 12288, 4096), (2048, 12288, 4096)])
def test_fused_gemm_llama7b_shapes(ops, M, N, K):
    """Full-size layer shapes: vs the fp32 product of the bit-exact dequantized weight (lga_q4_dequantize)."""
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    w = torch.randn(N, K, generator=g, device=DEV) * 0.02
    qw, sc = ops.quantize(w, 0, 128)
    wd = ops.q4_dequantize(qw, sc, N, K, 128, 0)
    x = torch.randn(M, K, generator=g, device=DEV).to(torch.bfloat16)
    res = torch.randn(M, N, generator=g, device=DEV).to(torch.bfloat16)
    y = ops.q4_gemm_fused(x, qw, sc, N, K, 128, 0, residual=res).float()
    h = x.float() @ wd.float().t()
    ref = h.to(torch.bfloat16).float() + res.float()
    err = (y - ref).abs() - (ref.abs() + h.abs()) * 2 ** -7
    assert float(err.max()) <= 2e-3
    # fc_1 || fc_2 + SwiGLU at the MLP shape
    if K == 4096 and N == 4096:
        I = 11008
        w1 = torch.randn(I, K, generator=g, device=DEV) * 0.02
        w2 = torch.randn(I, K, generator=g, device=DEV) * 0.02
        q1, s1 = ops.quantize(w1, 0, 128)
        q2, s2 = ops.quantize(w2, 0, 128)
        gg = ops.q4_gemm_swiglu(x, q1, s1, q2, s2, I, K, 128, 0).float()
        h1 = (x.float() @ ops.q4_dequantize(q1, s1, I, K, 128, 0).float().t()).to(torch.bfloat16)
        h2 = (x.float() @ ops.q4_dequantize(q2, s2, I, K, 128, 0).float().t()).to(torch.bfloat16)
        ref = ops.swiglu(h1.contiguous(), h2.contiguous()).float()
        assert float((gg - ref).abs().sub(_swiglu_tol(h1.float(), h2.float(), ref)).max()) <= 0.0


@pytest.mark.parametrize("M,N,K", [(17, 136, 256), (300, 392, 1024), (2048, 640, 4096)])
def test_fused_bf16_weights(ops, M, N, K):
    """fmt 2 (unquantized bf16 Linear, BASELINE config 2): the weight tile DMA'd as stored."""
    w = to_dev(bf16_np(_w(N, K, "bw")))
    x = to_dev(bf16_np(synth.normal((M, K), f"bwx{M}", 5, 1.0)))
    bias = to_dev(bf16_np(synth.normal((N,), "bwb", 5, 0.1)))
    y = ops.q4_gemm_fused(x, w, None, N, K, 64, 2, bias=bias).float()
    h = x.float() @ w.float().t() + bias.float()
    err = (y - h.to(torch.bfloat16).float()).abs() - h.abs() * 2 ** -7
    assert float(err.max()) <= 2e-3
    w2 = to_dev(bf16_np(_w(N, K, "bw2")))
    g = ops.q4_gemm_swiglu(x, w, None, w2, None, N, K, 64, 2).float()
    h1 = (x.float() @ w.float().t()).to(torch.bfloat16)
    h2 = (x.float() @ w2.float().t()).to(torch.bfloat16)
    ref = ops.swiglu(h1.contiguous(), h2.contiguous()).float()
    assert float((g - ref).abs().sub(_swiglu_tol(h1.float(), h2.float(), ref)).max()) <= 0.0


@pytest.mark.parametrize("M,N,K", [(64, 4096, 4096), (17, 4096, 11008), (128, 1024, 4096)])
def test_fused_gemm_split_k(ops, M, N, K, monkeypatch):
    """Short prompts split K over workgroups (fp32 slabs summed in slice order by the tile's last slice): the
    result is deterministic, within fp32 reassociation of the unsplit kernel, and within bf16 rounding of the
    fp32 product; also for the SwiGLU form."""
    g = torch.Generator(device=DEV).manual_seed(M * 7 + K)
    w = torch.randn(N, K, generator=g, device=DEV) * 0.02
    qw, sc = ops.quantize(w, 0, 128)
    x = torch.randn(M, K, generator=g, device=DEV).to(torch.bfloat16)
    assert ops.load_library().lga_q4f_workspace_bytes(M, N, K, 0) > 0  # this shape splits
    y1 = ops.q4_gemm_fused(x, qw, sc, N, K, 128, 0)
    y2 = ops.q4_gemm_fused(x, qw, sc, N, K, 128, 0)
    assert torch.equal(y1, y2), "split-K must be deterministic"
    monkeypatch.setenv("LGA_Q4F_SPLITS", "1")
    y0 = ops.q4_gemm_fused(x, qw, sc, N, K, 128, 0)
    monkeypatch.delenv("LGA_Q4F_SPLITS")
    h = x.float() @ ops.q4_dequantize(qw, sc, N, K, 128, 0).float().t()
    for y in (y0, y1):
        assert float(((y.float() - h).abs() - h.abs() * 2 ** -7).max()) <= 2e-3
    w2 = torch.randn(N, K, generator=g, device=DEV) * 0.02
    q2, s2 = ops.quantize(w2, 0, 128)
    gg = ops.q4_gemm_swiglu(x, qw, sc, q2, s2, N, K, 128, 0).float()
    h1 = h.to(torch.bfloat16)
    h2 = (x.float() @ ops.q4_dequantize(q2, s2, N, K, 128, 0).float().t()).to(torch.bfloat16)
    ref = ops.swiglu(h1.contiguous(), h2.contiguous()).float()
    assert float((gg - ref).abs().sub(_swiglu_tol(h1.float(), h2.float(), ref)).max()) <= 0.0


def test_fused_gemm_rejects_unsupported_shapes(ops):
    assert not ops.q4f_fits(16, 128, 96, 32, 0)   # K % 64
    assert not ops.q4f_fits(16, 132, 128, 64, 0)  # N % 8
    assert not ops.q4f_fits(16, 128, 128, 32, 0)  # group < 64
    x = torch.zeros(16, 96, dtype=torch.bfloat16, device=DEV)
    qw = torch.zeros(128, 48, dtype=torch.uint8, device=DEV)
    sc = torch.zeros(128, 3, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(RuntimeError, match="K % 64"):
        ops.q4_gemm_fused(x, qw, sc, 128, 96, 32, 0)


@pytest.mark.parametrize("fmt,group", [(0, 128), (1, 64), (3, 64)])
@pytest.mark.parametrize("M,N,K", [(300, 392, 1024), (513, 520, 768)])
def test_fused_gemm_256x256_tiles(ops, fmt, group, M, N, K, monkeypatch):
    """The 256 x 256 tile (64 x 128 outputs per wave, one K-step of prefetch; the planner picks it where its rounds
    fill the CUs better, e.g. fc_1 || fc_2 at 2048 tokens) forced on: plain with bias + residual, and SwiGLU."""
    monkeypatch.setenv("LGA_Q4F_BN", "256")
    w = _w(N, K, "bt")
    qw, sc, wd = _quant(ops, w, fmt, group)
    x = bf16_np(synth.normal((M, K), f"btx{M}x{K}", 5, 1.0))
    res = bf16_np(synth.normal((M, N), "btres", 5, 1.0))
    bias = bf16_np(synth.normal((N,), "btb", 5, 0.1))
    y = ops.q4_gemm_fused(to_dev(x), qw, sc, N, K, group, fmt, bias=to_dev(bias),
                          residual=to_dev(res)).float().cpu().numpy()
    h = x.astype(np.float64) @ wd.astype(np.float64).T + bias
    ref = bf16_np(h.astype(np.float32)) + res
    assert np.max(np.abs(y - ref) - (np.abs(ref) + np.abs(h)) * 2 ** -7) <= 2e-3
    w2 = _w(N, K, "bt2")
    q2, s2, d2 = _quant(ops, w2, fmt, group)
    g = ops.q4_gemm_swiglu(to_dev(x), qw, sc, q2, s2, N, K, group, fmt).float().cpu().numpy()
    h1 = x.astype(np.float64) @ wd.astype(np.float64).T
    h2 = x.astype(np.float64) @ d2.astype(np.float64).T
    a = bf16_np(h1.astype(np.float32))
    gref = bf16_np(bf16_np(_silu(a.astype(np.float64)).astype(np.float32)) * bf16_np(h2.astype(np.float32)))
    assert np.max(np.abs(g - gref) - _swiglu_tol(a, bf16_np(h2.astype(np.float32)), gref)) <= 0.0


@pytest.mark.parametrize("fmt", [0, 1, 3])
def test_fused_gemm_column_split(ops, fmt):
    """Long prompt, one wide matrix (the 7B qkv shape class): columns [0, 8192) run as a round of 256 x 256 tiles,
    the rest as 256 x 128 tiles — two launches over column ranges of one output (row stride N, offset weights /
    scales / bias / residual). Checked against the fp32 product of the bit-exact dequantized weight."""
    M, N, K = 2048, 12288, 1024
    group = 128 if fmt == 0 else 64
    g = torch.Generator(device=DEV).manual_seed(fmt + 5)
    w = torch.randn(N, K, generator=g, device=DEV) * 0.02
    qw, sc = ops.quantize(w, fmt, group)
    wd = ops.q4_dequantize(qw, sc, N, K, group, fmt)
    x = torch.randn(M, K, generator=g, device=DEV).to(torch.bfloat16)
    res = torch.randn(M, N, generator=g, device=DEV).to(torch.bfloat16)
    bias = (torch.randn(N, generator=g, device=DEV) * 0.1).to(torch.bfloat16)
    y = ops.q4_gemm_fused(x, qw, sc, N, K, group, fmt, bias=bias, residual=res).float()
    h = x.float() @ wd.float().t() + bias.float()
    ref = h.to(torch.bfloat16).float() + res.float()
    err = (y - ref).abs() - (ref.abs() + h.abs()) * 2 ** -7
    assert float(err.max()) <= 2e-3


@pytest.mark.parametrize("M,bn", [(1, None), (64, None), (128, None), (200, "128"), (200, "256")])
@pytest.mark.parametrize("splits", [2, 4, 8])
def test_fused_gemm_split_k_handoff_stress(ops, M, bn, splits, monkeypatch):
    """The split-K hand-off (csrc/gemm_q4f.hip: write-through sc1 slab stores, drain, barrier, a relaxed agent
    counter; the last slice reads the slabs with sc1 loads, no fences) across all four tile shapes (64 x 128,
    64 x 256, 256 x 128, 256 x 256) and 2 / 4 / 8 slices over many tiles: A, then B, then A again on the same slab
    workspace — a slab read that saw the previous call's partials would make the two A results differ or leave
    the fp32 product's rounding bound. Both the plain and the SwiGLU form."""
    N, K = 4096, 4096
    monkeypatch.setenv("LGA_Q4F_SPLITS", str(splits))
    if bn is not None:
        monkeypatch.setenv("LGA_Q4F_BN", bn)
    g = torch.Generator(device=DEV).manual_seed(M * 31 + splits)
    w = torch.randn(N, K, generator=g, device=DEV) * 0.02
    w2 = torch.randn(N, K, generator=g, device=DEV) * 0.02
    qw, sc = ops.quantize(w, 0, 128)
    q2, s2 = ops.quantize(w2, 0, 128)
    xa = torch.randn(M, K, generator=g, device=DEV).to(torch.bfloat16)
    xb = torch.randn(M, K, generator=g, device=DEV).to(torch.bfloat16) * 3
    ya = ops.q4_gemm_fused(xa, qw, sc, N, K, 128, 0)
    yb = ops.q4_gemm_fused(xb, qw, sc, N, K, 128, 0)
    ya2 = ops.q4_gemm_fused(xa, qw, sc, N, K, 128, 0)
    assert torch.equal(ya, ya2)
    wd = ops.q4_dequantize(qw, sc, N, K, 128, 0).float()
    for x, y in ((xa, ya), (xb, yb)):
        h = x.float() @ wd.t()
        assert float(((y.float() - h).abs() - h.abs() * 2 ** -7).max()) <= 2e-3
    ga = ops.q4_gemm_swiglu(xa, qw, sc, q2, s2, N, K, 128, 0)
    ops.q4_gemm_swiglu(xb, qw, sc, q2, s2, N, K, 128, 0)
    ga2 = ops.q4_gemm_swiglu(xa, qw, sc, q2, s2, N, K, 128, 0)
    assert torch.equal(ga, ga2)
    h1 = (xa.float() @ wd.t()).to(torch.bfloat16)
    h2 = (xa.float() @ ops.q4_dequantize(q2, s2, N, K, 128, 0).float().t()).to(torch.bfloat16)
    ref = ops.swiglu(h1.contiguous(), h2.contiguous()).float()
    assert float((ga.float() - ref).abs().sub(_swiglu_tol(h1.float(), h2.float(), ref)).max()) <= 0.0


# ------------------------------------------------------------------------------------------------ grouped MoE prefill
def _group_reference(ids: np.ndarray, E: int, bm: int):
    """CPU restatement of lga_moe_group: stable sort of the (token, slot) pairs by expert, m-tiles of bm rows."""
    T, k = ids.shape
    flat = ids.reshape(-1)
    order = np.argsort(flat, kind="stable")
    tiles, b = [], 0
    for e in range(E):
        c = int((flat == e).sum())
        for r in range(0, c, bm):
            tiles.append((e, b + r, min(bm, c - r)))
        b += c
    return tiles, (order // k).astype(np.int32), order.astype(np.int32)


@pytest.mark.parametrize("T,k,E,bm", [(1, 2, 8, 64), (37, 2, 8, 64), (300, 2, 8, 256), (2048, 2, 8, 256), (50, 3, 5, 64)])
def test_moe_group_table_matches_stable_sort(ops, T, k, E, bm):
    rng = np.random.default_rng(T * 7 + E)
    ids = np.stack([rng.choice(E, size=k, replace=False) for _ in range(T)]).astype(np.int32)
    tiles, xr, yr = ops.moe_group(torch.from_numpy(ids).to(DEV), E, bm)
    t_ref, xr_ref, yr_ref = _group_reference(ids, E, bm)
    tl = tiles.cpu().numpy()
    assert tl[0] == len(t_ref)
    assert [tuple(tl[1 + 3 * i: 4 + 3 * i]) for i in range(tl[0])] == t_ref
    assert np.array_equal(xr.cpu().numpy(), xr_ref) and np.array_equal(yr.cpu().numpy(), yr_ref)


@pytest.mark.parametrize("fmt,group", [(0, 128), (1, 64)])
@pytest.mark.parametrize("T", [5, 200, 700])
def test_grouped_expert_gemms_equal_per_expert_gemms(ops, fmt, group, T, monkeypatch):
    """The grouped prefill (fc_1 || fc_2 + SwiGLU over every expert's rows in one launch, then the grouped proj
    scattered to (token, slot)) against the per-expert fused GEMMs on gathered rows — the reference's loop
    (model.py:740-742) — bit for bit (no split-K on either side: each output's K-steps accumulate in order)."""
    monkeypatch.setenv("LGA_Q4F_SPLITS", "1")
    E, k, C, I = 4, 2, 512, 768
    rng = np.random.default_rng(T + fmt)
    ids = np.stack([rng.choice(E, size=k, replace=False) for _ in range(T)]).astype(np.int32)
    g0 = torch.Generator(device=DEV).manual_seed(T)
    q = {}
    for name, (N, K) in (("fc1", (I, C)), ("fc2", (I, C)), ("proj", (C, I))):
        ws = [ops.quantize(torch.randn(N, K, generator=g0, device=DEV) * 0.02, fmt, group) for _ in range(E)]
        q[name] = (torch.stack([w for w, _ in ws]), torch.stack([s for _, s in ws]))
    x = torch.randn(T, C, generator=g0, device=DEV).to(torch.bfloat16)
    rows, bm = T * k, ops.moe_grouped_bm(T * k)
    tiles, x_rows, y_rows = ops.moe_group(torch.from_numpy(ids).to(DEV), E, bm)
    g = ops.q4_gemm_swiglu_grouped(x, *q["fc1"], *q["fc2"], tiles, x_rows, rows, I, C, group, fmt, bm, E)
    eout = ops.q4_gemm_grouped(g, *q["proj"], tiles, y_rows, rows, C, I, group, fmt, bm, E).view(T, k, C)
    ref = torch.empty(T, k, C, dtype=torch.bfloat16, device=DEV)
    idt = torch.from_numpy(ids).to(DEV)
    for e in range(E):
        tok, slot = torch.where(idt == e)
        if tok.numel() == 0:
            continue
        xe = x.index_select(0, tok).contiguous()
        ge = ops.q4_gemm_swiglu(xe, q["fc1"][0][e], q["fc1"][1][e], q["fc2"][0][e], q["fc2"][1][e], I, C, group, fmt)
        ref[tok, slot] = ops.q4_gemm_fused(ge, q["proj"][0][e], q["proj"][1][e], C, I, group, fmt)
    assert torch.equal(eout, ref)
