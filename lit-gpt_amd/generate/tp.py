"""Tensor-parallel generation on the MI355X — drop-in for the reference's generate/tp.py.

Same sharding and semantics as /root/reference/generate/tp.py:28-92: qkv / fc_1 / fc_2 column-parallel (dim 0),
attn.proj / mlp.proj row-parallel (dim 1), bias split only for colwise (the reference's rowwise-bias behaviour is
kept), one all-reduce(sum) forward hook after attention and after the MLP, ``n_head``, ``n_embd``,
``n_query_groups`` divided by the world size (``ValueError`` when not divisible). Weights are sharded while
still float and quantized per shard afterwards (convert_module -> tensor_parallel -> to_device order,
generate/tp.py:171-190), block by block so a rank never holds the whole unsharded model. The collective for a
decode token is the xGMI one-shot all-reduce of lit_gpt/comm.py (graph-captured, fused with the Block residual
add); prefill messages use ``torch.distributed`` (backend "nccl" = RCCL over xGMI).

One process per GPU; launch with ``python -m torch.distributed.run --nproc-per-node N generate/tp.py ...``.
"""

from __future__ import annotations

import argparse
import os
import sys
import time
from functools import partial
from pathlib import Path
from typing import Optional, Union

import torch
import torch.distributed as dist

wd = Path(__file__).parent.parent.resolve()
if str(wd) not in sys.path:
    sys.path.append(str(wd))

import generate.base as generate_base  # noqa: E402
from lit_gpt import GPT, Config, comm  # noqa: E402
from lit_gpt.comm import all_reduce_output  # noqa: E402,F401  (the hook, reference generate/tp.py:73-74)
from lit_gpt.model import CausalSelfAttention, GptNeoxMLP, LLaMAMLP, LLaMAMoE  # noqa: E402


class Fabric:
    """The two attributes the sharding functions read from Lightning's Fabric (``world_size``, ``global_rank``)."""

    def __init__(self, world_size: int, global_rank: int) -> None:
        self.world_size, self.global_rank = world_size, global_rank


def tensor_parallel_linear(fabric, linear: torch.nn.Linear, style: str) -> None:
    world_size = fabric.world_size
    dim, attr = {"colwise": (0, "out_features"), "rowwise": (1, "in_features")}[style]
    size = getattr(linear, attr)
    if size % world_size != 0:
        raise ValueError(f"This linear's {attr} value ({size}) is not evenly divisible by the world size ({world_size})")
    shard = torch.tensor_split(linear.weight, world_size, dim=dim)[fabric.global_rank]
    linear.weight.data = shard
    setattr(linear, attr, shard.size(dim))
    if linear.bias is not None and dim == 0:
        bshard = torch.tensor_split(linear.bias, world_size)[fabric.global_rank]
        linear.bias = torch.nn.Parameter(bshard, requires_grad=linear.bias.requires_grad)


def tensor_parallel_mlp(fabric, mlp: Union[GptNeoxMLP, LLaMAMLP, LLaMAMoE]) -> None:
    if isinstance(mlp, LLaMAMLP):
        tensor_parallel_linear(fabric, mlp.fc_1, "colwise")
        tensor_parallel_linear(fabric, mlp.fc_2, "colwise")
        tensor_parallel_linear(fabric, mlp.proj, "rowwise")
        mlp.register_forward_hook(partial(all_reduce_output, fabric.world_size))
    elif isinstance(mlp, GptNeoxMLP):
        tensor_parallel_linear(fabric, mlp.fc, "colwise")
        tensor_parallel_linear(fabric, mlp.proj, "rowwise")
        mlp.register_forward_hook(partial(all_reduce_output, fabric.world_size))
    elif isinstance(mlp, LLaMAMoE):
        # expert slicing across ranks (as the reference)
        for expert in mlp.experts:
            tensor_parallel_mlp(fabric, expert)
    else:
        raise NotImplementedError


def tensor_parallel_attn(fabric, attn: CausalSelfAttention) -> None:
    tensor_parallel_linear(fabric, attn.attn, "colwise")
    tensor_parallel_linear(fabric, attn.proj, "rowwise")
    attn.register_forward_hook(partial(all_reduce_output, fabric.world_size))




def tensor_parallel(fabric, model: GPT) -> GPT:
    for block in model.transformer.h:
        tensor_parallel_block(fabric, block)
    return shard_config(fabric, model)


def tensor_parallel_block(fabric, block) -> None:
    """One block's share of ``tensor_parallel`` (build_model shards block by block, before quantizing)."""
    tensor_parallel_mlp(fabric, block.mlp)
    tensor_parallel_attn(fabric, block.attn)


def shard_config(fabric, model: GPT) -> GPT:
    """The config update at the end of the reference's ``tensor_parallel`` (generate/tp.py:84-91)."""
    world_size = fabric.world_size
    for attr in ("n_head", "n_embd", "n_query_groups"):
        size = getattr(model.config, attr)
        if size % world_size != 0:
            raise ValueError(f"This {attr} value ({size}) is not evenly divisible by the world size ({world_size})")
        setattr(model.config, attr, size // world_size)
    return model


def init_distributed(allreduce: Optional[str] = None) -> Fabric:
    """One process per GPU from the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*). With more
    than one rank the decode all-reduces go through the xGMI one-shot kernel (lit_gpt/comm.py) unless
    ``allreduce`` (or ``LGA_TP_ALLREDUCE``) is "rccl"; prefill messages always use RCCL."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for a one-GPU box (never set in production): every rank on cuda:0, gloo for the host-side
    # collectives (RCCL refuses two ranks on one device); the decode all-reduces stay on the xGMI kernel
    if os.environ.get("LGA_ONE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("LGA_DIST_BACKEND", "nccl")
    torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    mode = allreduce or os.environ.get("LGA_TP_ALLREDUCE", "xgmi")
    if mode not in ("xgmi", "rccl"):
        raise ValueError(f"allreduce must be 'xgmi' or 'rccl', got {mode!r}")
    if world > 1 and mode == "xgmi" and comm.get_default() is None:
        try:
            comm.set_default(comm.XgmiAllReduce(device=torch.device("cuda", local)))
        except comm.XgmiUnavailable as e:  # every rank gets here together: all stay on RCCL
            comm.fallback_reason = str(e)
            print(f"[generate/tp.py] xGMI one-shot all-reduce unavailable, decode all-reduces use RCCL: {e}",
                  file=sys.stderr)
    return Fabric(world, rank)


@torch.inference_mode()
def main(prompt: str = "What food do llamas eat?", *, num_samples: int = 1, max_new_tokens: int = 50,
         top_k: Optional[int] = 200, temperature: float = 0.8, checkpoint_dir: Path = Path("checkpoints"),
         quantize: Optional[str] = None, precision: Optional[str] = None, synthetic: Optional[str] = None,
         prompt_len: int = 16) -> None:
    fabric = init_distributed()
    device = torch.device("cuda", torch.cuda.current_device())
    if synthetic is not None:
        config = Config.from_name(synthetic)
        checkpoint_path = None
        g = torch.Generator(device="cpu").manual_seed(1234)
        encoded = torch.randint(0, config.vocab_size, (prompt_len,), generator=g, dtype=torch.int32).to(device)
        tokenizer = None
    else:
        from lit_gpt.tokenizer import Tokenizer

        config = Config.from_json(checkpoint_dir / "lit_config.json")
        checkpoint_path = checkpoint_dir / "lit_model.pth"
        tokenizer = Tokenizer(checkpoint_dir)
        encoded = tokenizer.encode(prompt, device=device)
    max_returned = encoded.size(0) + max_new_tokens
    t0 = time.perf_counter()
    model = generate_base.build_model(config, quantize=quantize, device=device, checkpoint_path=checkpoint_path,
                                      max_seq_length=max_returned, fabric=fabric)
    if fabric.world_size > 1:
        dist.barrier()
    if fabric.global_rank == 0:
        print(f"Time to load the model weights: {time.perf_counter() - t0:.02f} seconds.", file=sys.stderr)
    torch.manual_seed(1234)
    for i in range(num_samples):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        y = generate_base.generate(model, encoded, max_returned, temperature=temperature, top_k=top_k,
                                   eos_id=None if tokenizer is None else tokenizer.eos_id)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        for block in model.transformer.h:
            block.attn.kv_cache.reset_parameters()
        if fabric.global_rank == 0:
            print(tokenizer.decode(y) if tokenizer is not None else y.tolist())
            n = y.size(0) - encoded.size(0)
            print(f"Time for inference {i + 1}: {t:.02f} sec total, {n / t:.02f} tokens/sec", file=sys.stderr)


if __name__ == "__main__":
    p = argparse.ArgumentParser(description="Tensor-parallel generation")
    p.add_argument("--prompt", default="What food do llamas eat?")
    p.add_argument("--num_samples", type=int, default=1)
    p.add_argument("--max_new_tokens", type=int, default=50)
    p.add_argument("--top_k", type=int, default=200)
    p.add_argument("--temperature", type=float, default=0.8)
    p.add_argument("--checkpoint_dir", type=Path, default=Path("checkpoints"))
    p.add_argument("--quantize", default=None)
    p.add_argument("--precision", default=None)
    p.add_argument("--synthetic", default=None)
    p.add_argument("--prompt_len", type=int, default=16)
    a = p.parse_args()
    main(a.prompt, num_samples=a.num_samples, max_new_tokens=a.max_new_tokens, top_k=a.top_k,
         temperature=a.temperature, checkpoint_dir=a.checkpoint_dir, quantize=a.quantize, precision=a.precision,
         synthetic=a.synthetic, prompt_len=a.prompt_len)
