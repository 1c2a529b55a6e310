"""Streaming chat over the MI355X decode path — drop-in for the reference's chat/base.py.

Same functions and contract as /root/reference/chat/base.py: ``generate`` (:23-68) is a generator that yields
tokens as they are produced, holds back the last ``max(len(stop))`` tokens until they cannot begin a stop
sequence and returns without yielding a matched stop sequence; ``decode`` (:71-99) prints the stream
(token-by-token for HuggingFace tokenizers, re-decoding the prefix for sentencepiece) and returns the count;
``prompt_config`` (:191-365) for the model families this build runs (Llama-2 chat, CodeLlama / Mistral
instruct, plain — Mixtral-Instruct gets the plain template, as the reference's ``Mistral.*Instruct`` pattern gives); ``main`` (:102-188) is the interactive loop. MI355X difference: greedy chat
(``--temperature 0``) replays one HIP graph per token (lit_gpt/runtime.py ``DecodeGraph``) instead of
``torch.compile(mode="reduce-overhead")``.
"""

from __future__ import annotations

import argparse
import re
import sys
import time
from pathlib import Path
from typing import Iterator, List, Optional, Tuple

import torch

wd = Path(__file__).parent.parent.resolve()
if str(wd) not in sys.path:
    sys.path.append(str(wd))

from generate.base import SamplerRNG, build_model, graph_sampling, next_token  # noqa: E402
from lit_gpt import GPT, Config  # noqa: E402


def _tokens(model: GPT, prompt: torch.Tensor, n: int, temperature: float, top_k: Optional[int],
            use_graph: bool) -> Iterator[torch.Tensor]:
    """Up to ``n`` new tokens, one at a time: prefill at arange(T), then single-token steps."""
    T = prompt.size(0)
    rng = SamplerRNG(prompt.device) if temperature > 0.0 else None
    token = next_token(model, torch.arange(0, T, device=prompt.device), prompt.view(1, -1),
                       temperature=temperature, top_k=top_k, rng=rng).clone()
    yield token
    if n <= 1:
        return
    if use_graph and graph_sampling(model, temperature, top_k):
        from lit_gpt.runtime import DecodeGraph

        dg = DecodeGraph(model, token, T, temperature=temperature, top_k=top_k, rng=rng)
        yield dg.token.view(-1)[:1].clone()
        for _ in range(n - 2):
            yield dg.step().view(-1)[:1].clone()
        return
    input_pos = torch.tensor([T], device=prompt.device)
    for _ in range(n - 1):
        token = next_token(model, input_pos, token.view(1, -1), temperature=temperature, top_k=top_k,
                           rng=rng).clone()
        yield token
        input_pos = input_pos.add_(1)


@torch.inference_mode()
def generate(model: GPT, prompt: torch.Tensor, max_returned_tokens: int, *, temperature: float = 1.0,
             top_k: Optional[int] = None, stop_tokens: Tuple[List[int], ...] = (),
             use_graph: bool = True) -> Iterator[torch.Tensor]:
    """Continue ``prompt`` (shape (T,)) and yield the new tokens as they become safe to emit (reference
    :23-68): stop as soon as the generated tail equals one of ``stop_tokens``, never yielding that tail."""
    T = prompt.size(0)
    assert max_returned_tokens > T
    if model.max_seq_length < max_returned_tokens - 1:
        raise NotImplementedError(f"max_seq_length {model.max_seq_length} needs to be >= {max_returned_tokens - 1}")
    buffer_length = max((len(st) for st in stop_tokens), default=1)
    yield_i = 0
    tokens: List[torch.Tensor] = []
    ids: List[int] = []
    for t, token in enumerate(_tokens(model, prompt, max_returned_tokens - T, temperature, top_k, use_graph), 1):
        tokens.append(token)
        ids.append(int(token))
        if any(len(st) <= len(ids) and ids[-len(st):] == list(st) for st in stop_tokens):
            return
        if t - yield_i >= buffer_length:
            yield from tokens[yield_i:t]
            yield_i = t


def decode(tokenizer, token_stream: Iterator[torch.Tensor], out=None) -> int:
    """Print the stream as it arrives; returns the number of tokens printed (reference :71-99)."""
    out = out or sys.stdout
    n = 0
    if tokenizer.backend == "huggingface":
        try:
            for token in token_stream:
                print(tokenizer.decode(token), end="", flush=True, file=out)
                n += 1
        except KeyboardInterrupt:
            return n
    elif tokenizer.backend == "sentencepiece":
        # sentencepiece places spaces from the surrounding tokens: re-decode the prefix, print the new suffix
        so_far: List[int] = []
        decoded_so_far = ""
        try:
            for token in token_stream:
                so_far.extend(int(v) for v in token.view(-1).tolist())
                decoded_new = tokenizer.decode(torch.tensor(so_far, dtype=torch.long))
                print(decoded_new[len(decoded_so_far):], end="", flush=True, file=out)
                decoded_so_far = decoded_new
                n += 1
        except KeyboardInterrupt:
            return n
    else:
        raise NotImplementedError(tokenizer.backend)
    return n


_LLAMA2_SYSTEM = (
    "You are a helpful, respectful and honest assistant. Always answer as helpfully as possible, while being safe. "
    " Your answers should not include any harmful, unethical, racist, sexist, toxic, dangerous, or illegal content."
    " Please ensure that your responses are socially unbiased and positive in nature.\n\nIf a question does not make"
    " any sense, or is not factually coherent, explain why instead of answering something not correct. If you don't"
    " know the answer to a question, please don't share false information."
)


def prompt_config(checkpoint_dir: Path, tokenizer) -> Tuple[str, Tuple[List[int], ...]]:
    """System prompt template and stop sequences per checkpoint family (reference :191-365, the families whose
    blocks this build runs; anything else gets the reference's fallback ``"{prompt}"`` + eos)."""
    name = str(checkpoint_dir)
    eos = ([tokenizer.eos_id],)
    if re.search("Llama-2.*-chat", name):
        return f"[INST] <<SYS>>\n{_LLAMA2_SYSTEM}\n<</SYS>>\n\n {{prompt}} [/INST] ", eos
    if re.search("CodeLlama|Mistral.*Instruct", name):  # the reference's pattern: Mixtral-Instruct falls through
        return "<s>[INST] {prompt} [/INST]", eos
    return "{prompt}", eos


@torch.inference_mode()
def main(*, top_k: Optional[int] = 200, temperature: float = 0.8,
         checkpoint_dir: Path = Path("checkpoints/meta-llama/Llama-2-7b-chat-hf"),
         quantize: Optional[str] = None, precision: Optional[str] = None, compile: bool = False) -> None:
    precision = precision or "bf16-true"
    if precision != "bf16-true":
        raise NotImplementedError("the MI355X path computes in bf16 (precision bf16-true)")
    from lit_gpt.tokenizer import Tokenizer
    from lit_gpt.utils import check_valid_checkpoint_dir

    device = torch.device("cuda", torch.cuda.current_device())
    check_valid_checkpoint_dir(checkpoint_dir)
    config = Config.from_json(checkpoint_dir / "lit_config.json")
    checkpoint_path = checkpoint_dir / "lit_model.pth"
    print(f"Loading model {str(checkpoint_path)!r} with {config.__dict__}", file=sys.stderr)
    model = build_model(config, quantize=quantize, device=device, checkpoint_path=checkpoint_path)
    tokenizer = Tokenizer(checkpoint_dir)
    system_prompt, stop_tokens = prompt_config(checkpoint_dir, tokenizer)
    torch.manual_seed(1234)
    while True:
        try:
            prompt = input(">> Prompt: ")
        except (KeyboardInterrupt, EOFError):
            break
        if not prompt:
            break
        encoded = tokenizer.encode(system_prompt.format(prompt=prompt), device=device)
        y = generate(model, encoded, model.max_seq_length, temperature=temperature, top_k=top_k,
                     stop_tokens=stop_tokens)
        print(">> Reply: ", end="")
        t0 = time.perf_counter()
        n = decode(tokenizer, y)
        t = time.perf_counter() - t0
        for block in model.transformer.h:
            block.attn.kv_cache.reset_parameters()
        print(f"\nTime for inference: {t:.02f} sec total, {n / t:.02f} tokens/sec, {n} tokens", file=sys.stderr)
        print()


def _cli(argv=None) -> None:
    p = argparse.ArgumentParser(description="Starts a conversation with a tuned GPT model.")
    p.add_argument("--top_k", type=int, default=200)
    p.add_argument("--temperature", type=float, default=0.8)
    p.add_argument("--checkpoint_dir", type=Path, default=Path("checkpoints/meta-llama/Llama-2-7b-chat-hf"))
    p.add_argument("--quantize", default=None)
    p.add_argument("--precision", default=None)
    p.add_argument("--compile", action="store_true")
    a = p.parse_args(argv)
    main(top_k=a.top_k, temperature=a.temperature, checkpoint_dir=a.checkpoint_dir, quantize=a.quantize,
         precision=a.precision, compile=a.compile)


if __name__ == "__main__":
    _cli()
