"""Single-device generation on the MI355X — drop-in for the reference's generate/base.py.

Same functions and semantics as /root/reference/generate/base.py: ``multinomial_num_samples_1`` (:22-27),
``sample`` (:30-41), ``next_token`` (:44-47), ``generate`` (:50-93: prefill at ``arange(T)``, then one-token
steps at ``input_pos = T, T+1, ...``, stop on ``eos_id``, ``NotImplementedError`` when ``max_seq_length`` is too
short) and ``main`` (:96-187) with the same flags and the same stderr timing line. Differences:
  * greedy decoding (``temperature == 0``) and top-k sampling (``top_k`` <= 1024, the reference's default 200 at
    temperature 0.8) run each step as one HIP graph replay (lit_gpt/runtime.py) with the argmax / the fused
    top-k + softmax + inverse-CDF sampler on the device — the role ``--compile`` (CUDA graphs) plays in the
    reference; the sampler's uniforms come from a counter-based RNG seeded from torch's generator, so a seed
    reproduces a run but not the reference's exact torch.multinomial draws;
  * ``--quantize`` takes this build's formats (int4-g128, nf4 / bnb.nf4 / bnb.nf4-dq, bnb.fp4 / bnb.fp4-dq); without it the Linears
    stay bf16 ``nn.Linear`` (BASELINE config 2) and run on the bf16 GEMV / GEMM kernels;
  * ``--synthetic NAME`` builds a random-init model of a registered config (no checkpoint, no tokenizer): the
    prompt is ``--prompt_len`` synthetic token ids.
"""

from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path
from typing import Any, Optional

import torch

wd = Path(__file__).parent.parent.resolve()
if str(wd) not in sys.path:
    sys.path.append(str(wd))

from lit_gpt import GPT, Config  # noqa: E402
from lit_gpt import ops  # noqa: E402


def multinomial_num_samples_1(probs: torch.Tensor) -> torch.Tensor:
    return torch.multinomial(probs, num_samples=1)


class SamplerRNG:
    """State of the fused sampler's counter-based RNG (csrc/sample.hip): a 64-bit seed drawn from torch's default
    generator, so ``torch.manual_seed`` makes a run repeatable (generate/base.py:174), and a device counter the
    kernel advances once per draw, so a captured decode step draws a fresh uniform at every replay."""

    def __init__(self, device: torch.device, seed: Optional[int] = None) -> None:
        self.seed = int(torch.randint(0, 2**62, (1,))) if seed is None else int(seed)
        self.counter = torch.zeros(1, dtype=torch.int64, device=device)


def device_sampling(temperature: float, top_k: Optional[int], dtype: torch.dtype, vocab: int = 0) -> bool:
    """Whether ``sample`` at this setting runs as the one-launch HIP sampler (ops.sample_topk): temperature > 0 with
    top_k in [1, 1024] over bf16 logits of at most 65536 entries — the reference's defaults (top_k 200,
    temperature 0.8) included."""
    return (temperature > 0.0 and top_k is not None and 1 <= top_k <= ops.MAX_TOP_K and dtype == torch.bfloat16
            and vocab <= ops.MAX_SAMPLE_VOCAB)


def sample(logits: torch.Tensor, temperature: float = 1.0, top_k: Optional[int] = None,
           rng: Optional[SamplerRNG] = None) -> torch.Tensor:
    """logits (1, T, V) on the GPU -> (1,) token (generate/base.py:30-41). Greedy runs the HIP argmax (lowest index
    on ties; top-k cannot change the arg-max); temperature > 0 with top_k <= 1024 over bf16 logits runs the HIP
    top-k + softmax + inverse-CDF sampler in one launch (``rng`` carries its RNG state; a fresh one is drawn from
    torch's generator when omitted); other settings follow the reference's torch ops, softmax in the logits' dtype."""
    logits = logits[0, -1]
    if not logits.is_cuda:
        raise RuntimeError("sample: logits must be on the GPU (this build has no CPU path)")
    if temperature > 0.0:
        if device_sampling(temperature, top_k, logits.dtype, logits.size(-1)):
            rng = rng if rng is not None else SamplerRNG(logits.device)
            return ops.sample_topk(logits.contiguous(), top_k, temperature, seed=rng.seed, counter=rng.counter)
        if top_k is not None:
            v, i = torch.topk(logits, min(top_k, logits.size(-1)))
            logits = torch.full_like(logits, float("-inf")).scatter_(-1, i, v)
        probs = torch.nn.functional.softmax(logits / temperature, dim=-1)
        return multinomial_num_samples_1(probs)
    return ops.argmax((logits if logits.dtype == torch.float32 else logits.to(torch.bfloat16)).contiguous())


def next_token(model: GPT, input_pos: torch.Tensor, x: torch.Tensor, **kwargs: Any) -> torch.Tensor:
    logits = model(x, input_pos, last_token_only=True)
    return sample(logits, **kwargs).to(dtype=x.dtype)


def graph_sampling(model: GPT, temperature: float, top_k: Optional[int]) -> bool:
    """Whether decode steps at this setting run as captured HIP graphs (lit_gpt/runtime.py DecodeGraph): greedy, or
    the device sampler (``device_sampling``) over the model's bf16 logits."""
    wte = model.transformer.wte.weight
    return temperature == 0.0 or device_sampling(temperature, top_k, wte.dtype, model.config.padded_vocab_size)


DECODE_CHUNK = 8  # greedy decode steps per graph launch (lit_gpt/runtime.py DecodeGraph.steps)


@torch.inference_mode()
def generate(model: GPT, prompt: torch.Tensor, max_returned_tokens: int, *, temperature: float = 1.0,
             top_k: Optional[int] = None, eos_id: Optional[int] = None, use_graph: bool = True) -> torch.Tensor:
    """Takes a conditioning sequence (prompt, shape (T,)) and continues it; returns (T + new,) ids."""
    T = prompt.size(0)
    assert max_returned_tokens > T
    if model.max_seq_length < max_returned_tokens - 1:
        raise NotImplementedError(f"max_seq_length {model.max_seq_length} needs to be >= {max_returned_tokens - 1}")
    device = prompt.device
    tokens = [prompt]
    rng = SamplerRNG(device) if temperature > 0.0 else None
    token = next_token(model, torch.arange(0, T, device=device), prompt.view(1, -1), temperature=temperature,
                       top_k=top_k, rng=rng).clone()
    tokens.append(token)
    n_steps = max_returned_tokens - T - 1
    if n_steps <= 0:
        return torch.cat(tokens)
    if use_graph and graph_sampling(model, temperature, top_k):
        from lit_gpt.runtime import DecodeGraph

        # (the prefill's token is never tested against eos: the reference's loop only tests the decoded ones,
        # generate/base.py:86-92)
        # runs the first decode step eagerly, then captures the step (and DECODE_CHUNK steps as one graph)
        dg = DecodeGraph(model, token, T, chunk=DECODE_CHUNK if n_steps > DECODE_CHUNK else 1,
                         temperature=temperature, top_k=top_k, rng=rng)
        out = torch.empty(n_steps, dtype=prompt.dtype, device=device)
        out[0] = dg.token.view(-1)[0]
        produced = 1
        if not (eos_id is not None and int(out[0]) == eos_id):
            i = 1
            while i < n_steps:
                if dg.chunk > 1 and n_steps - i >= dg.chunk:
                    out[i:i + dg.chunk] = dg.steps()
                    n = dg.chunk
                else:
                    out[i] = dg.step().view(-1)[0]
                    n = 1
                produced = i + n
                if eos_id is not None:  # one host check per launch; tokens past an eos are dropped
                    hit = (out[i:i + n] == eos_id).nonzero()
                    if hit.numel():
                        produced = i + int(hit[0]) + 1
                        break
                i += n
        tokens.append(out[:produced])
        _check_collectives()
        return torch.cat(tokens)
    input_pos = torch.tensor([T], device=device)
    for _ in range(n_steps):
        token = next_token(model, input_pos, token.view(1, -1), temperature=temperature, top_k=top_k,
                           rng=rng).clone()
        tokens.append(token)
        if eos_id is not None and int(token) == eos_id:
            break
        input_pos = input_pos.add_(1)
    _check_collectives()
    return torch.cat(tokens)


def _check_collectives() -> None:
    """Under tensor parallelism with the xGMI all-reduce: raise (on every rank) if any decode all-reduce of this
    run gave up waiting for a peer — its logits were summed from partial data (lit_gpt/comm.py check_errors)."""
    from lit_gpt import comm

    if comm.get_default() is not None:
        comm.check_errors()


def build_model(config: Config, *, quantize: Optional[str], device: torch.device, seed: int = 1234,
                checkpoint_path: Optional[Path] = None, max_seq_length: Optional[int] = None,
                fabric=None, rope_positions: str = "reference", prefill_rows: Optional[int] = None,
                dtype: torch.dtype = torch.bfloat16) -> GPT:
    """Instantiate on the meta device, then materialise (load, or random-init as GPT._init_weights) the float
    weights on the GPU in the model's parameter order; with ``fabric`` (world_size / global_rank, generate/tp.py)
    every block is sharded (``tensor_parallel_block``) and quantized as soon as its weights exist, so a rank holds
    at most one unsharded block (70B TP=8: ~1.7 GB, not the whole 138 GB model). Then the rope tables and the KV
    cache. Mirrors generate/base.py:151-171 / generate/tp.py:157-190 (convert_module -> tensor_parallel ->
    to_device: the values each rank quantizes are its float shard, as there).

    ``rope_positions="reference"`` builds the rope tables under a bf16 default dtype, as the reference's
    ``with fabric.init_tensor(): model.max_seq_length = ...`` does under bf16-true / bnb precision
    (generate/base.py:153-157): positions above 256 round to bf16. ``"exact"`` keeps fp32 positions.
    ``prefill_rows`` (the prompt length about to be served) is accepted for API stability; the prefill GEMMs are
    hand-written (csrc/gemm_q4f.hip) and need no per-shape tuning or warm-up. ``dtype`` float32 is the reference's
    ``--precision 32-true`` (GPT-NeoX family, csrc/fp32.hip; no quantization, no TP)."""
    if dtype not in (torch.bfloat16, torch.float32):
        raise NotImplementedError(f"precision with dtype {dtype}: the MI355X path computes in bf16 or fp32")
    if dtype == torch.float32 and (quantize is not None or (fabric is not None and fabric.world_size > 1)):
        raise NotImplementedError("32-true runs unquantized on one device (BASELINE config 1)")
    if rope_positions not in ("reference", "exact"):
        raise ValueError(f"rope_positions must be 'reference' or 'exact', got {rope_positions!r}")
    from lit_gpt.quantize import QuantizedPrecision

    if quantize is not None:
        from lit_gpt.quantize import parse_mode

        parse_mode(quantize)  # unsupported modes fail before any weight is materialised
    tp = None
    if fabric is not None and fabric.world_size > 1:
        from generate import tp

        for attr in ("n_head", "n_embd", "n_query_groups"):  # fail before materialising (generate/tp.py:87-90)
            if getattr(config, attr) % fabric.world_size:
                raise ValueError(f"This {attr} value ({getattr(config, attr)}) is not evenly divisible by the world "
                                 f"size ({fabric.world_size})")
    with torch.device("meta"):
        model = GPT(config)
    state = None
    if checkpoint_path is not None:
        state = torch.load(str(checkpoint_path), mmap=True, map_location="cpu", weights_only=True)
        state = state.get("model", state)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    precision = QuantizedPrecision(quantize) if quantize is not None else None

    def finish(module: torch.nn.Module) -> None:
        """Shard (TP) and quantize one fully materialised block (or the top-level Linears)."""
        if tp is not None and hasattr(module, "attn"):
            tp.tensor_parallel_block(fabric, module)
        if precision is not None:
            precision.convert_module(module, device)
            mlp = getattr(module, "mlp", None)
            if hasattr(mlp, "_stack"):  # sparse MoE: the experts' packed weights stacked now, not in the first prompt
                mlp._stack()
        else:  # bf16-true: the Linears stay nn.Linear; TP row shards are strided views -> own contiguous storage
            for mod in module.modules():
                if isinstance(mod, torch.nn.Linear) and not mod.weight.is_contiguous():
                    mod.weight = torch.nn.Parameter(mod.weight.data.contiguous(), requires_grad=False)

    open_block = None
    for name, p in list(model.named_parameters()):
        mod_name, _, attr = name.rpartition(".")
        parts = name.split(".")
        blk = int(parts[2]) if parts[:2] == ["transformer", "h"] else None
        if open_block is not None and blk != open_block:
            finish(model.transformer.h[open_block])
        open_block = blk
        mod = model.get_submodule(mod_name)
        if state is not None:
            t = state[name].to(device=device, dtype=dtype)
        elif attr == "weight" and (isinstance(mod, (torch.nn.Linear, torch.nn.Embedding))):
            t = torch.empty(p.shape, dtype=torch.float32, device=device).normal_(0.0, 0.02, generator=gen)
            t = t.to(dtype)
        elif attr == "bias":
            t = torch.zeros(p.shape, dtype=dtype, device=device)
        else:  # norm weights
            t = torch.ones(p.shape, dtype=dtype, device=device)
        setattr(mod, attr, torch.nn.Parameter(t, requires_grad=False))
    if open_block is not None:
        finish(model.transformer.h[open_block])
    if precision is not None:  # lm_head (replicated under TP, as the reference leaves it unsharded)
        precision.convert_module(model, device)
    if tp is not None:
        tp.shard_config(fabric, model)
    torch.cuda.empty_cache()
    prev = torch.get_default_dtype()
    # (32-true: the reference's default dtype stays float32, so its positions are exact)
    torch.set_default_dtype(torch.bfloat16 if rope_positions == "reference" and dtype == torch.bfloat16
                            else torch.float32)
    try:
        model.max_seq_length = max_seq_length or config.block_size
        model.cos, model.sin = model.rope_cache(device=device)
    finally:
        torch.set_default_dtype(prev)
    model.set_kv_cache(batch_size=1, device=device, dtype=dtype)
    ops.preload_kernels()  # the runtime would otherwise build each prefill kernel inside the first prompt
    return model.eval()


@torch.inference_mode()
def main(prompt: str = "What food do llamas eat?", *, num_samples: int = 1, max_new_tokens: int = 50,
         top_k: Optional[int] = 200, temperature: float = 0.8,
         checkpoint_dir: Path = Path("checkpoints/stabilityai/stablelm-base-alpha-3b"),
         quantize: Optional[str] = None, precision: Optional[str] = None, compile: bool = False,
         synthetic: Optional[str] = None, prompt_len: int = 16) -> None:
    precision = precision or "bf16-true"
    if precision not in ("bf16-true", "32-true"):
        raise NotImplementedError("the MI355X path computes in bf16 (bf16-true) or fp32 (32-true)")
    dtype = torch.float32 if precision == "32-true" else torch.bfloat16
    device = torch.device("cuda", torch.cuda.current_device())
    tokenizer = None
    if synthetic is not None:
        config = Config.from_name(synthetic)
        checkpoint_path = None
        g = torch.Generator(device="cpu").manual_seed(1234)
        encoded = torch.randint(0, config.vocab_size, (prompt_len,), generator=g, dtype=torch.int32).to(device)
    else:
        from lit_gpt.tokenizer import Tokenizer
        from lit_gpt.utils import check_valid_checkpoint_dir

        check_valid_checkpoint_dir(checkpoint_dir)
        config = Config.from_json(checkpoint_dir / "lit_config.json")
        checkpoint_path = checkpoint_dir / "lit_model.pth"
        tokenizer = Tokenizer(checkpoint_dir)
        encoded = tokenizer.encode(prompt, device=device)
    prompt_length = encoded.size(0)
    max_returned_tokens = prompt_length + max_new_tokens
    print(f"Loading model {str(checkpoint_path or synthetic)!r} with {config.__dict__}", file=sys.stderr)
    t0 = time.perf_counter()
    model = build_model(config, quantize=quantize, device=device, checkpoint_path=checkpoint_path,
                        max_seq_length=max_returned_tokens, prefill_rows=prompt_length, dtype=dtype)
    print(f"Time to load the model weights: {time.perf_counter() - t0:.02f} seconds.", file=sys.stderr)
    torch.manual_seed(1234)
    eos_id = tokenizer.eos_id if tokenizer is not None else None
    for i in range(num_samples):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        y = generate(model, encoded, max_returned_tokens, temperature=temperature, top_k=top_k, eos_id=eos_id)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        for block in model.transformer.h:
            block.attn.kv_cache.reset_parameters()
        print(tokenizer.decode(y) if tokenizer is not None else y.tolist())
        tokens_generated = y.size(0) - prompt_length
        print(f"Time for inference {i + 1}: {t:.02f} sec total, {tokens_generated / t:.02f} tokens/sec",
              file=sys.stderr)
    print(f"Memory used: {torch.cuda.max_memory_allocated() / 1e9:.02f} GB", file=sys.stderr)


def _cli(argv=None) -> None:
    p = argparse.ArgumentParser(description="Generates text samples based on a pre-trained model and tokenizer.")
    p.add_argument("--prompt", default="What food do llamas eat?")
    p.add_argument("--num_samples", type=int, default=1)
    p.add_argument("--max_new_tokens", type=int, default=50)
    p.add_argument("--top_k", type=int, default=200)
    p.add_argument("--temperature", type=float, default=0.8)
    p.add_argument("--checkpoint_dir", type=Path, default=Path("checkpoints/stabilityai/stablelm-base-alpha-3b"))
    p.add_argument("--quantize", default=None)
    p.add_argument("--precision", default=None)
    p.add_argument("--compile", action="store_true")
    p.add_argument("--synthetic", default=None, help="random-init model of this registered config name")
    p.add_argument("--prompt_len", type=int, default=16)
    a = p.parse_args(argv)
    main(a.prompt, num_samples=a.num_samples, max_new_tokens=a.max_new_tokens, top_k=a.top_k,
         temperature=a.temperature, checkpoint_dir=a.checkpoint_dir, quantize=a.quantize, precision=a.precision,
         compile=a.compile, synthetic=a.synthetic, prompt_len=a.prompt_len)


if __name__ == "__main__":
    _cli()
