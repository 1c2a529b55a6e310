"""Layer placement across the GPUs of one process — drop-in for the reference's generate/sequentially.py.

Same functions and contract as /root/reference/generate/sequentially.py: ``sequential`` (:30-77, balanced
partitioning only, ``NotImplementedError`` otherwise), ``layer_to_device`` (:80-86), ``move_block_input``
(:89-92), ``move_block_output`` (:95-97), ``replace_device`` (:100-114, ``ValueError`` on a submodule split over
devices) and ``main`` (:117-223) with its flags and stderr lines. MI355X differences:
  * the model is built and quantized on the root GPU (the device quantizer, lit_gpt/quantize.py) and each
    block's packed weights are then moved to its GPU — 288 GB of HBM per MI355X holds any registered model's
    weights on the root during the hand-out, so no CPU staging copy is made;
  * every block on a non-root GPU runs with that GPU as the current HIP device (the C-ABI launches on
    ``torch.cuda.current_stream()``), so its kernels land on its own stream;
  * ``device_ids`` (optional) maps partition i to a device index; the default is partition i -> GPU i as in
    the reference. Tests use it to run two partitions on one GPU with the hooks active;
  * greedy generation replays one HIP graph per step when every partition sits on one GPU; across GPUs it runs
    eagerly (the reference likewise cannot use CUDA graphs across device indices, :206-208).
"""

from __future__ import annotations

import argparse
import itertools
import sys
import time
from collections import OrderedDict
from functools import partial
from pathlib import Path
from typing import Optional, Sequence, Type

import torch

wd = Path(__file__).parent.parent.resolve()
if str(wd) not in sys.path:
    sys.path.append(str(wd))

import generate.base as generate_base  # noqa: E402
from lit_gpt import GPT, Config  # noqa: E402
from lit_gpt.model import Block, CausalMask, KVCache  # noqa: E402


@torch.inference_mode()
def sequential(model: GPT, root: torch.device, max_seq_length: int, devices: int,
               device_ids: Optional[Sequence[int]] = None) -> GPT:
    """Place ``n_layer / devices`` consecutive blocks on each device, build each block's KV cache there and
    install the hooks that carry activations across partition boundaries (reference :30-77)."""
    if model.config.n_layer % devices:
        raise NotImplementedError(
            f"Only balanced partitioning is implemented: n_layer={model.config.n_layer}, devices {devices}")
    if device_ids is None:
        device_ids = list(range(devices))
    if len(device_ids) != devices:
        raise ValueError(f"device_ids has {len(device_ids)} entries for {devices} devices")
    root = torch.device(root)
    layers_per_rank = model.config.n_layer // devices
    mapping = layer_to_device(model, chunk_on=Block, chunk_size=layers_per_rank)
    rope_len = model.cos.size(-1) if model.cos is not None and model.cos.device.type != "meta" else None

    for path, part in mapping.items():
        block = model.get_submodule(path)
        target = _device(root, device_ids[part])
        print(f"Moving {path!r} to {target}", file=sys.stderr)
        replace_device(block, replace=root, by=target)
        replace_device(block, replace=torch.device("cpu"), by=target)
        block.attn.kv_cache = block.attn.build_kv_cache(1, max_seq_length, rope_len, target)

    # odd ends on the root (reference :55-60): the rope tables are rebuilt under the caller's default dtype — the
    # reference rebuilds them under ``with root:`` only, outside fabric.init_tensor, so positions stay fp32
    model.max_seq_length = max_seq_length
    model.cos, model.sin = model.rope_cache(device=root)
    model.mask_cache = CausalMask(max_seq_length, root)  # reference sequentially.py:58 builds the tensor; no kernel reads it
    for name, sub in model.named_modules():
        if isinstance(sub, Block) or any(name.startswith(p + ".") for p in mapping):
            continue
        replace_device(sub, replace=torch.device("cpu"), by=root)

    # one copy of the rope tables per GPU, made here: the blocks' input hook substitutes it for the root tables
    # instead of copying max_seq x n_elem fp32 twice per block per token
    replicas = {}
    for path, part in mapping.items():
        target = _device(root, device_ids[part])
        if part > 0 and target not in replicas:
            replicas[target] = {_tensor_key(t): t.to(target) for t in (model.cos, model.sin)}

    for layer_num, (path, part) in enumerate(mapping.items()):
        block = model.get_submodule(path)
        target = _device(root, device_ids[part])
        if part > 0:
            # inputs (x, cos, sin, mask, input_pos) follow the block; the block runs with its GPU current
            block.register_forward_pre_hook(partial(_use_replicas, replicas[target]))
            block.register_forward_pre_hook(partial(move_block_input, target))
            block.register_forward_pre_hook(partial(_enter_device, target))
            block.register_forward_hook(partial(_leave_device, root))
        if layer_num == model.config.n_layer - 1 and devices > 1:
            block.register_forward_hook(partial(move_block_output, root))
    return model


def _device(root: torch.device, index: int) -> torch.device:
    return torch.device(root.type, index) if root.type != "cpu" else root


def layer_to_device(module: torch.nn.Module, chunk_on: Type[torch.nn.Module],
                    chunk_size: int) -> "OrderedDict[str, int]":
    """Block path -> partition index, in definition (= execution) order (reference :80-86)."""
    hits = [name for name, sub in module.named_modules() if isinstance(sub, chunk_on)]
    return OrderedDict((name, i // chunk_size) for i, name in enumerate(hits))


def _tensor_key(t: torch.Tensor):
    return (t.device, t.data_ptr(), tuple(t.shape), t.dtype)


def _use_replicas(replicas, module: torch.nn.Module, ins):
    """``forward_pre_hook``: swap inputs that are the root's rope tables for this block's device copy (a table
    rebuilt since ``sequential`` ran no longer matches and is copied by ``move_block_input`` as before)."""
    return tuple(replicas.get(_tensor_key(t), t) if isinstance(t, torch.Tensor) else t for t in ins)


def move_block_input(device: torch.device, module: torch.nn.Module, ins):
    """``forward_pre_hook``: move a Block's tensor inputs to its device (None stays None; reference :89-92)."""
    return tuple(t.to(device) if isinstance(t, torch.Tensor) else t for t in ins)


def move_block_output(device: torch.device, module: torch.nn.Module, ins, outs) -> torch.Tensor:
    """``forward_hook``: move the last Block's output back to the root device (reference :95-97)."""
    return outs.to(device)


def _enter_device(device: torch.device, module: torch.nn.Module, ins) -> None:
    if device.type == "cuda":
        torch.cuda.set_device(device)


def _leave_device(root: torch.device, module: torch.nn.Module, ins, outs) -> None:
    if root.type == "cuda":
        torch.cuda.set_device(root)


def replace_device(module: torch.nn.Module, replace: torch.device, by: torch.device) -> torch.nn.Module:
    """Move every submodule whose own tensors all sit on ``replace`` to ``by`` (reference :100-114). KV caches
    are rebuilt by ``sequential`` and skipped here."""
    replace, by = torch.device(replace), torch.device(by)
    for name, sub in module.named_modules():
        if isinstance(sub, KVCache):
            continue
        tensors = dict(itertools.chain(sub.named_parameters(recurse=False), sub.named_buffers(recurse=False)))
        if not tensors:
            continue
        devices = {t.device for t in tensors.values()}
        if len(devices) != 1:
            path_to_device = {f"{name}.{p}": t.device for p, t in tensors.items()}
            raise ValueError(f"Found multiple devices: {path_to_device}")
        if _same(devices.pop(), replace):
            sub.to(by)
    return module


def _same(a: torch.device, b: torch.device) -> bool:
    if a.type != b.type:
        return False
    if a.type != "cuda":
        return True
    ia = a.index if a.index is not None else torch.cuda.current_device()
    ib = b.index if b.index is not None else torch.cuda.current_device()
    return ia == ib


@torch.inference_mode()
def main(prompt: str = "What food do llamas eat?", *, num_samples: int = 1, max_new_tokens: int = 50,
         top_k: Optional[int] = 200, temperature: float = 0.8,
         checkpoint_dir: Path = Path("checkpoints/mistralai/Mistral-7B-Instruct-v0.1"),
         quantize: Optional[str] = None, precision: Optional[str] = None, compile: bool = False,
         synthetic: Optional[str] = None, prompt_len: int = 16, devices: Optional[int] = None) -> None:
    precision = precision or "bf16-true"
    if precision != "bf16-true":
        raise NotImplementedError("the MI355X path computes in bf16 (precision bf16-true)")
    if compile:
        raise NotImplementedError  # as the reference (:180-182); greedy decode uses HIP graphs on one device
    total_devices = devices or torch.cuda.device_count()
    print(f"Using {total_devices} devices", file=sys.stderr)
    root = torch.device("cuda", 0)
    tokenizer = None
    if synthetic is not None:
        config = Config.from_name(synthetic)
        checkpoint_path = None
        g = torch.Generator(device="cpu").manual_seed(1234)
        encoded = torch.randint(0, config.vocab_size, (prompt_len,), generator=g, dtype=torch.int32).to(root)
    else:
        from lit_gpt.tokenizer import Tokenizer
        from lit_gpt.utils import check_valid_checkpoint_dir

        check_valid_checkpoint_dir(checkpoint_dir)
        config = Config.from_json(checkpoint_dir / "lit_config.json")
        checkpoint_path = checkpoint_dir / "lit_model.pth"
        tokenizer = Tokenizer(checkpoint_dir)
        encoded = tokenizer.encode(prompt, device=root)
    prompt_length = encoded.size(0)
    max_returned_tokens = prompt_length + max_new_tokens
    print(f"Loading model {str(checkpoint_path or synthetic)!r} with {config.__dict__}", file=sys.stderr)
    t0 = time.perf_counter()
    model = generate_base.build_model(config, quantize=quantize, device=root, checkpoint_path=checkpoint_path,
                                      max_seq_length=max_returned_tokens)
    print(f"Time to load the model weights: {time.perf_counter() - t0:.02f} seconds.", file=sys.stderr)
    t0 = time.perf_counter()
    model = sequential(model, root, max_returned_tokens, total_devices)
    print(f"Time to sequential-ize the model: {time.perf_counter() - t0:.02f} seconds.", file=sys.stderr)
    torch.manual_seed(1234)
    eos_id = tokenizer.eos_id if tokenizer is not None else None
    for i in range(num_samples):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        y = generate_base.generate(model, encoded, max_returned_tokens, temperature=temperature, top_k=top_k,
                                   eos_id=eos_id, use_graph=total_devices == 1)
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
    p = argparse.ArgumentParser(description="Generates text with the blocks spread over the node's GPUs.")
    p.add_argument("--prompt", default="What food do llamas eat?")
    p.add_argument("--num_samples", type=int, default=1)
    p.add_argument("--max_new_tokens", type=int, default=50)
    p.add_argument("--top_k", type=int, default=200)
    p.add_argument("--temperature", type=float, default=0.8)
    p.add_argument("--checkpoint_dir", type=Path, default=Path("checkpoints/mistralai/Mistral-7B-Instruct-v0.1"))
    p.add_argument("--quantize", default=None)
    p.add_argument("--precision", default=None)
    p.add_argument("--compile", action="store_true")
    p.add_argument("--synthetic", default=None, help="random-init model of this registered config name")
    p.add_argument("--prompt_len", type=int, default=16)
    p.add_argument("--devices", type=int, default=None, help="partitions (default: every visible GPU)")
    a = p.parse_args(argv)
    main(a.prompt, num_samples=a.num_samples, max_new_tokens=a.max_new_tokens, top_k=a.top_k,
         temperature=a.temperature, checkpoint_dir=a.checkpoint_dir, quantize=a.quantize, precision=a.precision,
         compile=a.compile, synthetic=a.synthetic, prompt_len=a.prompt_len, devices=a.devices)


if __name__ == "__main__":
    _cli()
