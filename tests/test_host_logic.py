"""Host-side logic on the CPU: Config, TP sharding (known answers from the reference), hook placement, gloo TP."""

import os
import socket
from dataclasses import replace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import model as om
from oracle import synth
from oracle.tp import shard_linear


def test_config_derived_fields_match_reference():
    from lit_gpt import Config

    c = Config.from_name("Llama-2-7b-hf")
    assert (c.n_layer, c.n_head, c.n_embd, c.n_query_groups, c.head_size) == (32, 32, 4096, 32, 128)
    assert (c.padded_vocab_size, c.intermediate_size, c.rope_n_elem, c.block_size) == (32000, 11008, 128, 4096)
    c = Config.from_name("Llama-2-70b-chat-hf")
    assert (c.n_query_groups, c.head_size, c.intermediate_size) == (8, 128, 28672)
    c = Config.from_name("Mixtral-8x7B-v0.1")
    assert (c.n_expert, c.n_expert_per_token, c.rope_base, c.block_size, c.padded_vocab_size) == (8, 2, 1000000, 32768, 32000)
    c = Config.from_name("pythia-160m")
    assert (c.padded_vocab_size, c.rope_n_elem, c.intermediate_size) == (50304, 16, 3072)
    with pytest.raises(ValueError, match="not a supported config"):
        Config.from_name("nope")
    with pytest.raises(ValueError, match="intermediate_size"):
        Config(_mlp_class="LLaMAMLP")


def test_config_from_json_and_checkpoint(tmp_path):
    import json

    from lit_gpt import Config

    (tmp_path / "lit_config.json").write_text(json.dumps(
        {"name": "x", "org": "me", "block_size": 128, "vocab_size": 50, "n_layer": 2, "n_head": 4, "n_embd": 8,
         "condense_ratio": 2}))
    c = Config.from_json(tmp_path / "lit_config.json")
    assert c.hf_config == {"name": "x", "org": "me"} and c.rope_condense_ratio == 2 and c.padded_vocab_size == 512
    assert Config.from_checkpoint(tmp_path).n_layer == 2
    with pytest.raises(FileNotFoundError):
        Config.from_checkpoint(tmp_path / "missing")


def test_tensor_parallel_linear_known_answers(golden):
    """Same known answers as the reference's tests/test_generate_tp.py:14-40 and golden g4."""
    from generate.tp import Fabric, tensor_parallel_linear

    def get_linear(bias=True):
        lin = torch.nn.Linear(8, 8, bias=bias)
        lin.weight.data = torch.arange(64, dtype=torch.float32).reshape(8, 8)
        if bias:
            lin.bias.data = torch.arange(8, dtype=torch.float32)
        return lin

    lin = get_linear()
    tensor_parallel_linear(Fabric(4, 2), lin, "colwise")
    torch.testing.assert_close(lin.weight, torch.arange(32, 48, dtype=torch.float32).reshape(2, 8))
    torch.testing.assert_close(lin.bias, torch.arange(4, 6, dtype=torch.float32))
    lin = get_linear(bias=False)
    tensor_parallel_linear(Fabric(4, 2), lin, "rowwise")
    e = torch.arange(4, 62, 8, dtype=torch.float32).reshape(8, 1)
    torch.testing.assert_close(lin.weight, torch.cat([e, e + 1], dim=1))
    g = golden("g4_tp.npz")
    for world in (2, 4, 8):
        for rank in range(world):
            for style in ("colwise", "rowwise"):
                key = f"w{world}_r{rank}_{style}"
                lin = torch.nn.Linear(16, 24, bias=True)
                lin.weight.data = torch.arange(24 * 16, dtype=torch.float32).reshape(24, 16)
                lin.bias.data = torch.arange(24, dtype=torch.float32)
                if f"{key}_error" in g:
                    with pytest.raises(ValueError):
                        tensor_parallel_linear(Fabric(world, rank), lin, style)
                    continue
                tensor_parallel_linear(Fabric(world, rank), lin, style)
                np.testing.assert_array_equal(lin.weight.detach().numpy(), g[f"{key}_weight"])
                np.testing.assert_array_equal(lin.bias.detach().numpy(), g[f"{key}_bias"])


@pytest.mark.parametrize("name", ["Llama-2-70b-hf", "Mixtral-8x7B-v0.1"])
def test_tensor_parallel_hook_placement(name):
    """tests/test_generate_tp.py:43-103 analogue: hooks on attn and mlp (per expert for MoE), config / 8."""
    from generate.tp import Fabric, tensor_parallel
    from lit_gpt import GPT

    with torch.device("meta"):
        model = GPT.from_name(name, n_layer=3, n_expert=2)
    config = replace(model.config)
    tensor_parallel(Fabric(8, 1), model)
    hooks = {}
    for n, m in model.named_modules():
        for h in m._forward_hooks.values():
            hooks.setdefault(n, []).append((h.func.__name__, h.args))
    if name.startswith("Mixtral"):
        expected = {f"transformer.h.{i}.{s}" for i in range(3) for s in ("attn", "mlp.experts.0", "mlp.experts.1")}
    else:
        expected = {f"transformer.h.{i}.{s}" for i in range(3) for s in ("attn", "mlp")}
    assert set(hooks) == expected
    assert all(v == [("all_reduce_output", (8,))] for v in hooks.values())
    assert model.config.n_embd * 8 == config.n_embd and model.config.n_head * 8 == config.n_head
    assert model.config.n_query_groups * 8 == config.n_query_groups


def test_tensor_parallel_divisibility_error():
    from generate.tp import Fabric, tensor_parallel
    from lit_gpt import GPT

    with torch.device("meta"):
        model = GPT.from_name("Llama-2-7b-hf", n_layer=1)
    with pytest.raises(ValueError, match="not evenly divisible"):
        tensor_parallel(Fabric(3, 0), model)


# ---------------------------------------------------------------------------------------- gloo, world_size 2
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tp_worker(rank, world, port, q):
    """Each rank shards the float weights exactly as generate/tp.py does, computes its partial attention/MLP
    outputs with the oracle's math and sums them with the same all_reduce_output hook function (gloo here,
    RCCL on the GPU); logits must equal the single-process model."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from generate.tp import Fabric, all_reduce_output
        from lit_gpt import Config

        cfg = Config.from_name("Llama-2-70b-hf", n_layer=2, n_embd=256, n_head=4, n_query_groups=2,
                               intermediate_size=512, vocab_size=500, padding_multiple=64, block_size=64)
        sd = synth.state_dict(cfg, seed=3)
        f = Fabric(world, rank)
        local = dict(sd)
        for i in range(cfg.n_layer):
            p = f"transformer.h.{i}"
            for name, style in (("attn.attn", "colwise"), ("attn.proj", "rowwise"), ("mlp.fc_1", "colwise"),
                                ("mlp.fc_2", "colwise"), ("mlp.proj", "rowwise")):
                local[f"{p}.{name}.weight"], _ = shard_linear(sd[f"{p}.{name}.weight"], None, style, world, rank)
        lcfg = replace(cfg)
        lcfg.n_head, lcfg.n_embd, lcfg.n_query_groups = cfg.n_head // world, cfg.n_embd // world, cfg.n_query_groups // world
        lcfg.head_size = cfg.head_size
        m = om.OracleGPT(lcfg, local)
        m.cfg.n_embd = cfg.n_embd  # residual stream keeps the full width

        orig_attn, orig_mlp = m._attn, m._mlp
        m._attn = lambda *a: all_reduce_output(world, None, None, orig_attn(*a).contiguous())
        m._mlp = lambda *a: all_reduce_output(world, None, None, orig_mlp(*a).contiguous())
        m.set_kv_cache(20)
        ids = torch.from_numpy(synth.token_ids(12, cfg.vocab_size, seed=3))
        out = [m.forward(ids[:8], torch.arange(8))[-1]]
        for t in range(8, 12):
            out.append(m.forward(ids[t:t + 1], torch.tensor([t]))[-1])
        if rank == 0:
            q.put(torch.stack(out).numpy())
    finally:
        dist.destroy_process_group()


def test_tp2_gloo_matches_single_process():
    from lit_gpt import Config

    cfg = Config.from_name("Llama-2-70b-hf", n_layer=2, n_embd=256, n_head=4, n_query_groups=2,
                           intermediate_size=512, vocab_size=500, padding_multiple=64, block_size=64)
    m = om.OracleGPT(cfg, synth.state_dict(cfg, seed=3))
    m.set_kv_cache(20)
    ids = torch.from_numpy(synth.token_ids(12, cfg.vocab_size, seed=3))
    ref = [m.forward(ids[:8], torch.arange(8))[-1]]
    for t in range(8, 12):
        ref.append(m.forward(ids[t:t + 1], torch.tensor([t]))[-1])
    ref = torch.stack(ref).numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    np.testing.assert_allclose(got, ref, rtol=0, atol=2e-5)


def test_rope_cache_follows_reference_default_dtype(golden):
    """build_rope_cache takes its positions in the default dtype like the reference (lit_gpt/model.py:758): fp32
    positions by default, bf16-rounded positions under a bf16 default (the reference's init_tensor context)."""
    from lit_gpt.model import build_rope_cache

    g = golden("g3_ops.npz")
    for dt, tag in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
        prev = torch.get_default_dtype()
        torch.set_default_dtype(dt)
        try:
            cos, sin = build_rope_cache(2304, 128)
        finally:
            torch.set_default_dtype(prev)
        assert cos.dtype == torch.float32
        np.testing.assert_array_equal(cos[2040:2050].numpy(), g[f"rope_cos_{tag}"])
        np.testing.assert_array_equal(sin[2040:2050].numpy(), g[f"rope_sin_{tag}"])
    cos, _ = build_rope_cache(64, 16, base=1000000, condense_ratio=2)
    np.testing.assert_array_equal(cos.numpy(), g["rope_small_cos"])


def test_product_rope_long_context_rows_match_reference(golden):
    """The product's build_rope_cache at 4k-32k positions, base 1e4 and 1e6, fp32 and bf16 default dtype: bit-equal
    to the reference's tables (tests/golden/g5_rope_long.npz, make_golden_rope.py)."""
    from lit_gpt.model import build_rope_cache

    g = golden("g5_rope_long.npz")
    rows = g["rows"]
    for base in (10000, 1000000):
        for dt, tag in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
            prev = torch.get_default_dtype()
            torch.set_default_dtype(dt)
            try:
                cos, sin = build_rope_cache(32768, 128, base=base)
            finally:
                torch.set_default_dtype(prev)
            np.testing.assert_array_equal(cos[rows].numpy(), g[f"cos_{base}_{tag}"])
            np.testing.assert_array_equal(sin[rows].numpy(), g[f"sin_{base}_{tag}"])


def test_topk_order_restatement_matches_cpu_torch_topk():
    """oracle.model.topk_order (the spec of lga_moe_route) == torch.topk on the CPU, ties included."""
    import random

    from oracle.model import topk_order

    rng = random.Random(7)
    for _ in range(4000):
        n = rng.choice([8, 8, 4, 6, 7, 5, 3, 2])
        k = rng.randint(1, n)
        pool = rng.choice([[0.0, 1.0, 2.0], [0.0, -0.0, 1.0, 1.5], [float(x) for x in range(5)], None])
        vals = [rng.gauss(0, 1) if pool is None else rng.choice(pool) for _ in range(n)]
        t = torch.tensor(vals, dtype=torch.bfloat16).view(1, -1)
        assert topk_order(t[0].float().tolist(), k) == torch.topk(t, k).indices[0].tolist(), (vals, k)


def test_decode_attention_split_heuristic_per_tp_rank():
    """Sequence splits chosen for T = 1 attention (ops.decode_splits): 8 for Llama-2-7B's 32 groups, at most 16 for
    the few groups a tensor-parallel rank keeps, 32 for caches of >= 12k rows (measured on MI355X,
    tools/attn_sweep.py)."""
    from lit_gpt import ops

    assert ops.decode_splits(32, 1, 128, 2304) == 8  # 7B TP=1
    assert ops.decode_splits(16, 1, 128, 2304) == 16  # 7B TP=2
    assert ops.decode_splits(4, 1, 128, 2304) == 16  # 7B TP=8 (was 64: 10.9 vs 7.8 us)
    assert ops.decode_splits(1, 8, 128, 2304) == 16  # 70B TP=8: one KV group, 8 heads per group
    assert ops.decode_splits(4, 4, 128, 32768) == 32  # Mixtral TP=2 at 32k context (long caches: up to 32)
    assert ops.decode_splits(8, 4, 128, 32068) == 32  # Mixtral TP=1, 32k prompt
    assert ops.decode_splits(8, 4, 128, 12287) == 16
    assert ops.decode_splits(32, 1, 128, 32768) == 8  # 7B at 32k: one workgroup per CU already
    assert ops.decode_splits(4, 1, 128, 64) == 4  # short caches: >= 16 keys per split


def test_double_quant_code_table_is_bitsandbytes_dynamic_map():
    """The product's 256-entry code for bnb.nf4-dq (lit_gpt/quantize.py) equals the oracle's restatement of
    bitsandbytes create_dynamic_map(signed=True) bit for bit, and the mode parses as nf4 blocks of 64."""
    import numpy as np

    from lit_gpt import ops
    from lit_gpt.quantize import bnb_dynamic_map, parse_mode
    from oracle import quant

    assert np.array_equal(bnb_dynamic_map("cpu").numpy(), quant.dynamic_map())
    assert parse_mode("bnb.nf4-dq") == (ops.FMT_NF4, 64)
    a = np.linspace(0.01, 0.2, 1000, dtype=np.float32)
    q, amax2, off, out = quant.double_quant_absmax(a)
    assert q.dtype == np.uint8 and amax2.shape == (4,) and np.abs(out - a).max() <= 0.01 * a.max()



def test_fp4_oracle_is_bitsandbytes_fp4():
    """oracle/quant.py's bnb.fp4 restatement: the code table is bitsandbytes get_4bit_type('fp4') (= the values
    dDequantizeFP4Tree returns), every pivot sits halfway between neighbouring magnitudes, quantize picks the
    nearest code (ties to the smaller magnitude), dequantize -> quantize is idempotent, and the modes parse as
    fp4 blocks of 64 on the nf4 kernels' table slot."""
    import numpy as np

    from lit_gpt import ops
    from lit_gpt.quantize import parse_mode
    from oracle import quant

    tree = {0: 0.0, 1: 5.208333333e-03, 2: 0.66666667, 3: 1.0, 4: 0.33333333, 5: 0.5, 6: 0.16666667, 7: 0.25}
    for c, v in tree.items():
        assert quant.FP4[c] == np.float32(v) and quant.FP4[c + 8] == -np.float32(v)
    assert np.signbit(quant.FP4[8])
    mags = np.sort(quant.FP4[:8])
    np.testing.assert_allclose(quant.FP4_PIVOTS, (mags[1:] + mags[:-1]) / 2, rtol=2e-6)
    assert list(quant.FP4[quant.FP4_CODE_OF_RANK]) == list(mags)
    rng = np.random.default_rng(7)
    w = rng.standard_normal((8, 256)).astype(np.float32)
    p, a = quant.quantize_fp4(w, 64)
    d = quant.dequantize_fp4(p, a, 64)
    xn = w.reshape(8, 4, 64) / a[..., None]
    err = np.abs(d.reshape(8, 4, 64) / a[..., None] - xn)
    nearest = np.abs(np.abs(xn)[..., None] - mags).min(-1)
    assert np.all(err <= nearest + 1e-6)
    np.testing.assert_array_equal(quant.dequantize_fp4(*quant.quantize_fp4(d, 64), 64), d)
    assert parse_mode("bnb.fp4") == (ops.FMT_FP4, 64) and parse_mode("bnb.fp4-dq") == (ops.FMT_FP4, 64)


def test_oracle_route_override_hook():
    """OracleGPT.route_override (the MoE parity tests' near-tie adoption): an override returning the oracle's own
    expert sets leaves the logits bit-identical, and one that swaps a token's set changes only what it routes."""
    from lit_gpt import Config

    cfg = Config.from_name("Mixtral-8x7B-v0.1", n_layer=1, n_embd=128, n_head=4, n_query_groups=2,
                           intermediate_size=96, vocab_size=200, padding_multiple=64, block_size=64)
    sd = synth.state_dict(cfg, seed=3)
    idx = torch.from_numpy(synth.token_ids(6, cfg.vocab_size, seed=3))
    base = om.OracleGPT(cfg, sd, dtype=torch.float64)
    base.set_kv_cache(16)
    want = base.forward(idx, torch.arange(6))
    same = om.OracleGPT(cfg, sd, dtype=torch.float64)
    same.set_kv_cache(16)
    seen = []
    same.route_override = lambda router, i: (seen.append(i.clone()), i)[1]
    assert torch.equal(same.forward(idx, torch.arange(6)), want)
    assert len(seen) == cfg.n_layer and seen[0].shape == (6, cfg.n_expert_per_token)
    other = om.OracleGPT(cfg, sd, dtype=torch.float64)
    other.set_kv_cache(16)

    def swap_last(router, i):
        j = i.clone()
        j[-1] = torch.topk(router[-1], cfg.n_expert_per_token + 1).indices[1:]  # 2nd and 3rd best
        return j

    other.route_override = swap_last
    got = other.forward(idx, torch.arange(6))
    assert torch.equal(got[:-1], want[:-1]) and not torch.equal(got[-1], want[-1])
