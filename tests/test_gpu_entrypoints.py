"""GPU tests for the remaining inference entry points over the same kernels: generate/sequentially.py (layer
placement; reference tests/test_generate_sequentially.py) and chat/base.py streaming (reference
tests/test_chat.py). Outputs must be token-identical to generate/base.py's on the same weights AND follow the CPU
oracle (the restatement of the reference, teacher-forced on the produced tokens) wherever its margin is clear."""

import pytest
import torch

from oracle import synth
from test_gpu_model import DEV, _cfg, assert_tokens_follow_oracle, build_gpu_model

pytestmark = pytest.mark.gpu


def _reset(model):
    for b in model.transformer.h:
        b.attn.kv_cache.reset_parameters()


@pytest.mark.parametrize("key,mode,parts", [("mha", "int4-g128", 2), ("mqa", "int4-g128", 3),
                                            ("moe", "int4-g128", 2), ("gqa", "bf16", 2)])
@pytest.mark.parametrize("use_graph", [True, False])
@torch.inference_mode()
def test_sequential_partitions_match_single_device(key, mode, parts, use_graph):
    from generate.base import generate
    from generate.sequentially import sequential

    cfg = _cfg(key)
    sd = synth.state_dict(cfg, seed=41)
    T, N = 16, 20
    prompt = torch.from_numpy(synth.token_ids(T, cfg.vocab_size, seed=41)).to(DEV)
    model = build_gpu_model(cfg, sd, mode, T + N)
    y_ref = generate(model, prompt, T + N, temperature=0.0, use_graph=use_graph).cpu()
    _reset(model)
    # every partition on cuda:0 (one GPU on the test box): the boundary hooks run, the blocks' KV caches are
    # rebuilt per partition, the rope tables and mask are rebuilt on the root
    model = sequential(model, DEV, T + N, parts, device_ids=[0] * parts)
    hooked = [b for b in model.transformer.h if b._forward_pre_hooks]
    assert len(hooked) == cfg.n_layer - cfg.n_layer // parts
    y = generate(model, prompt, T + N, temperature=0.0, use_graph=use_graph).cpu()
    assert torch.equal(y, y_ref)
    assert assert_tokens_follow_oracle(cfg, sd, mode, prompt.cpu(), y) >= N // 4


@torch.inference_mode()
def test_chat_stream_matches_generate_and_stops():
    from chat.base import generate as chat_generate
    from generate.base import generate

    cfg = _cfg("gqa")
    sd = synth.state_dict(cfg, seed=43)
    T, N = 12, 16
    prompt = torch.from_numpy(synth.token_ids(T, cfg.vocab_size, seed=43)).to(DEV)
    model = build_gpu_model(cfg, sd, "int4-g128", T + N)
    y = generate(model, prompt, T + N, temperature=0.0).cpu()
    new = [int(v) for v in y[T:]]
    assert assert_tokens_follow_oracle(cfg, sd, "int4-g128", prompt.cpu(), y) >= N // 4
    for use_graph in (True, False):
        _reset(model)
        got = [int(t) for t in chat_generate(model, prompt, T + N, temperature=0.0, use_graph=use_graph)]
        assert got == new  # buffer of 1 token: every token is yielded as soon as it is produced
        # a two-token stop sequence taken from the stream: the yield schedule of reference chat/base.py:55-66
        _reset(model)
        stop = (new[5:7],)
        got = [int(t) for t in chat_generate(model, prompt, T + N, temperature=0.0, stop_tokens=stop,
                                             use_graph=use_graph)]
        assert got == _reference_schedule(new, stop)
        assert len(got) < 7


def _reference_schedule(produced, stop_tokens):
    """Plain-Python restatement of the reference's stop/buffer loop (chat/base.py:53-66)."""
    buf = max((len(s) for s in stop_tokens), default=1)
    out, yield_i, toks = [], 0, []
    for t, v in enumerate(produced, 1):
        toks.append(v)
        if any(len(s) <= len(toks) and toks[-len(s):] == list(s) for s in stop_tokens):
            return out
        if t - yield_i >= buf:
            out += toks[yield_i:t]
            yield_i = t
    return out


@torch.inference_mode()
def test_converted_hf_checkpoint_generates_same_tokens(tmp_path, monkeypatch):
    """HF-layout shards -> scripts/convert_hf_checkpoint.py -> generate/base.py's loader: the same greedy tokens
    as the model built straight from the lit-layout weights."""
    from safetensors.torch import save_file

    import scripts.convert_hf_checkpoint as cth
    from generate.base import build_model, generate
    from lit_gpt import Config
    from test_convert_hf_checkpoint import _hf_state

    cfg = _cfg("gqa")
    sd = synth.state_dict(cfg, seed=47)
    lit = {k: torch.from_numpy(v) for k, v in sd.items()}
    save_file({k: v.contiguous() for k, v in _hf_state(cfg, lit).items()}, str(tmp_path / "model.safetensors"))
    name, kw = "Llama-2-70b-hf", dict(n_layer=2, n_embd=1024, n_head=8, n_query_groups=2, intermediate_size=512,
                                      vocab_size=1000, padding_multiple=64, block_size=256)

    class TinyConfig(Config):
        @classmethod
        def from_name(cls, n, **k):
            return Config.from_name(n, **kw)

    monkeypatch.setattr(cth, "Config", TinyConfig)
    cth.convert_hf_checkpoint(checkpoint_dir=tmp_path, model_name=name)
    T, N = 16, 12
    prompt = torch.from_numpy(synth.token_ids(T, cfg.vocab_size, seed=47)).to(DEV)
    ref_model = build_gpu_model(cfg, sd, "int4-g128", T + N)
    y_ref = generate(ref_model, prompt, T + N, temperature=0.0).cpu()
    del ref_model
    loaded_cfg = Config.from_json(tmp_path / "lit_config.json")
    model = build_model(loaded_cfg, quantize="int4-g128", device=DEV, checkpoint_path=tmp_path / "lit_model.pth",
                        max_seq_length=T + N, rope_positions="exact")
    y = generate(model, prompt, T + N, temperature=0.0).cpu()
    assert torch.equal(y, y_ref)
