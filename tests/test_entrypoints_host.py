"""CPU tests of the host logic of generate/sequentially.py and chat/base.py (reference
tests/test_generate_sequentially.py: layer_to_device, replace_device; tests/test_chat.py: stop-token
buffering) — no kernels run."""

import pytest
import torch


def _tiny(n_layer=6):
    from lit_gpt import GPT, Config

    cfg = Config.from_name("Llama-2-7b-hf", n_layer=n_layer, n_embd=64, n_head=4, intermediate_size=96,
                           vocab_size=100, padding_multiple=64, block_size=32)
    with torch.device("meta"):
        return GPT(cfg)


@pytest.mark.parametrize("n_layer,chunk,expected", [(6, 3, [0, 0, 0, 1, 1, 1]), (6, 2, [0, 0, 1, 1, 2, 2]),
                                                    (4, 1, [0, 1, 2, 3])])
def test_layer_to_device(n_layer, chunk, expected):
    from generate.sequentially import layer_to_device
    from lit_gpt.model import Block

    m = layer_to_device(_tiny(n_layer), chunk_on=Block, chunk_size=chunk)
    assert list(m) == [f"transformer.h.{i}" for i in range(n_layer)]
    assert list(m.values()) == expected


def test_sequential_unbalanced_raises():
    from generate.sequentially import sequential

    with pytest.raises(NotImplementedError, match="Only balanced partitioning"):
        sequential(_tiny(6), torch.device("cpu"), 32, 4)


def test_replace_device():
    from generate.sequentially import replace_device

    class Sub(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.register_buffer("a", torch.zeros(2, device="meta"))
            self.b = torch.nn.Parameter(torch.zeros(2))

    m = torch.nn.Sequential(torch.nn.Linear(2, 2), torch.nn.Linear(2, 2, device="meta"))
    replace_device(m, replace=torch.device("cpu"), by=torch.device("meta"))
    assert all(p.device.type == "meta" for p in m.parameters())
    with pytest.raises(ValueError, match="multiple devices"):
        replace_device(Sub(), replace=torch.device("cpu"), by=torch.device("meta"))


def test_move_block_hooks_keep_none():
    from generate.sequentially import move_block_input, move_block_output

    x = torch.ones(1, 1, 4)
    out = move_block_input(torch.device("cpu"), None, (x, None, torch.zeros(2)))
    assert out[1] is None and torch.equal(out[0], x)
    assert torch.equal(move_block_output(torch.device("cpu"), None, (), x), x)


def _run_chat(monkeypatch, produced, stop, max_new):
    import chat.base as cb

    class FakeModel:
        max_seq_length = 1000

    def fake_tokens(model, prompt, n, temperature, top_k, use_graph):
        for v in produced[:n]:
            yield torch.tensor([v])

    monkeypatch.setattr(cb, "_tokens", fake_tokens)
    prompt = torch.zeros(3, dtype=torch.int64)
    return [int(t) for t in cb.generate(FakeModel(), prompt, 3 + max_new, stop_tokens=stop)]


def test_chat_stop_tokens(monkeypatch):
    # reference tests/test_chat.py semantics: tokens are held back until they cannot start a stop sequence;
    # a matched stop sequence is never yielded; without a match the loop ends at max_returned_tokens
    assert _run_chat(monkeypatch, [1, 2, 3, 4, 5], (), 5) == [1, 2, 3, 4, 5]
    assert _run_chat(monkeypatch, [1, 2, 3, 4, 5], ([3],), 5) == [1, 2]
    assert _run_chat(monkeypatch, [1, 2, 3, 4, 5], ([3, 4],), 5) == [1, 2]
    assert _run_chat(monkeypatch, [1, 2, 3, 4, 5], ([9, 9],), 5) == [1, 2, 3, 4]  # buffered tail not flushed
    # the buffer flushes in whole chunks of max(len(stop)) (reference chat/base.py:61-66): [3, 2] is released at
    # step 4, before step 5 completes the stop sequence [2, 5] — the reference's own behaviour, kept as is
    assert _run_chat(monkeypatch, [1, 2, 3, 2, 5, 6], ([2, 5], [9]), 6) == [1, 2, 3, 2]
    assert _run_chat(monkeypatch, [1, 2, 5, 6], ([2, 5],), 4) == [1, 2]


def test_chat_prompt_config():
    from pathlib import Path

    from chat.base import prompt_config

    class Tok:
        eos_id = 2

    sp, stop = prompt_config(Path("checkpoints/meta-llama/Llama-2-7b-chat-hf"), Tok())
    assert sp.startswith("[INST] <<SYS>>\n") and sp.endswith(" {prompt} [/INST] ") and stop == ([2],)
    sp, stop = prompt_config(Path("checkpoints/mistralai/Mistral-7B-Instruct-v0.1"), Tok())
    assert sp == "<s>[INST] {prompt} [/INST]"
    # the reference's regex (chat/base.py:326) does not match Mixtral: plain template
    assert prompt_config(Path("checkpoints/mistralai/Mixtral-8x7B-Instruct-v0.1"), Tok()) == ("{prompt}", ([2],))
    assert prompt_config(Path("checkpoints/meta-llama/Llama-2-7b-hf"), Tok()) == ("{prompt}", ([2],))


def test_sampling_route_and_rng_state():
    """generate/base.py's sample() routing (reference :30-41): the reference's default (top_k 200, temperature 0.8)
    and any top_k in [1, 1024] over bf16 logits go to the one-launch device sampler (and so into the decode graph);
    top_k None / > 1024, fp32 logits and greedy do not. SamplerRNG draws its seed from torch's generator, so
    torch.manual_seed reproduces a run, and keeps a device counter starting at zero."""
    from generate.base import SamplerRNG, device_sampling

    bf, f32 = torch.bfloat16, torch.float32
    assert device_sampling(0.8, 200, bf)
    assert device_sampling(1.0, 1, bf) and device_sampling(1.0, 1024, bf)
    assert not device_sampling(0.8, None, bf)
    assert not device_sampling(0.8, 1025, bf)
    assert not device_sampling(0.8, 0, bf)
    assert not device_sampling(0.8, 200, f32)
    assert not device_sampling(0.0, 200, bf)
    assert device_sampling(0.8, 200, bf, 65536) and not device_sampling(0.8, 200, bf, 65537)
    torch.manual_seed(1234)
    a = SamplerRNG(torch.device("cpu"))
    torch.manual_seed(1234)
    b = SamplerRNG(torch.device("cpu"))
    c = SamplerRNG(torch.device("cpu"))
    assert a.seed == b.seed != c.seed
    assert a.counter.dtype == torch.int64 and int(a.counter) == 0
    assert SamplerRNG(torch.device("cpu"), seed=7).seed == 7


def test_sample_refuses_cpu_logits():
    from generate.base import sample

    with pytest.raises(RuntimeError):
        sample(torch.zeros(1, 1, 10), temperature=0.8, top_k=5)
