"""Worker for tests/test_gpu_model.py::test_tensor_parallel_2_ranks_one_gpu (launched by torch.distributed.run).

Both ranks share cuda:0 and the `gloo` backend (RCCL needs one GPU per rank; the driver's multi-GPU bench covers
RCCL itself): the point is the sharding + all-reduce hooks + per-shard quantization + HIP kernels on real shard
shapes. Rank 0 also runs the unsharded model and writes both logit sequences to argv[1].
"""

import os
import sys
from dataclasses import replace
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]

from generate import tp as gtp  # noqa: E402
from lit_gpt import GPT, Config  # noqa: E402
from lit_gpt.quantize import QuantizedPrecision  # noqa: E402
from oracle import synth  # noqa: E402

DEV = torch.device("cuda", 0)


def build(cfg, sd, mode, fabric=None):
    model = GPT(cfg)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    if fabric is not None:
        gtp.tensor_parallel(fabric, model)
    model = model.to(device=DEV, dtype=torch.bfloat16)
    if mode != "bf16":  # "bf16": the shards stay nn.Linear (bf16 GEMV / GEMM kernels)
        QuantizedPrecision(mode).convert_module(model, DEV)
    model.max_seq_length = 64
    model.set_kv_cache(1, device=DEV)
    return model.eval()


@torch.inference_mode()
def run(model, ids):
    """Logits per step, and per step the smallest router gap between the k-th and (k+1)-th expert (MoE only;
    +inf for dense blocks): a step whose gap is within a few bf16 ulps may route differently under TP."""
    gaps = []
    for blk in model.transformer.h:
        if hasattr(blk.mlp, "gate"):
            k = model.config.n_expert_per_token

            def hook(m, a, o, k=k):
                v = torch.sort(o.float().reshape(-1, o.size(-1)), dim=-1, descending=True).values
                gaps.append(float((v[:, k - 1] - v[:, k]).min()))

            blk.mlp.gate.register_forward_hook(hook)
    out, step_gap = [], []

    def step(logits):
        out.append(logits[0, -1].float())
        step_gap.append(min(gaps, default=float("inf")))
        gaps.clear()

    step(model(ids[:8].view(1, -1), torch.arange(8, device=DEV)))
    for i in range(8, ids.numel()):
        step(model(ids[i:i + 1].view(1, 1), torch.tensor([i], device=DEV)))
    return torch.stack(out).cpu().numpy(), np.array(step_gap)


def main():
    out_path, mode = sys.argv[1], sys.argv[2]
    family = sys.argv[3] if len(sys.argv) > 3 else "llama"
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    if family == "moe":  # generate/tp.py:58-62: experts sliced, gate replicated, all-reduce per expert output
        cfg = Config.from_name("Mixtral-8x7B-v0.1", n_layer=2, n_embd=1024, n_head=8, n_query_groups=4,
                               intermediate_size=1024, vocab_size=1000, padding_multiple=64, block_size=256)
    else:
        cfg = Config.from_name("Llama-2-70b-hf", n_layer=2, n_embd=1024, n_head=8, n_query_groups=4,
                               intermediate_size=1024, vocab_size=1000, padding_multiple=64, block_size=256)
    sd = synth.state_dict(cfg, seed=11)
    ids = torch.from_numpy(synth.token_ids(16, cfg.vocab_size, seed=5)).to(torch.int32).to(DEV)
    tp_logits, _ = run(build(replace(cfg), sd, mode, gtp.Fabric(world, rank)), ids)
    dist.barrier()
    if rank == 0:
        ref_logits, gaps = run(build(cfg, sd, mode), ids)
        np.savez(out_path, tp=tp_logits, ref=ref_logits, gaps=gaps)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
