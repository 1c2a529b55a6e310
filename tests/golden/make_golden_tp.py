"""G4 tensor-parallel logits: the REFERENCE's own ``tensor_parallel`` (/root/reference/generate/tp.py:28-92, its
forward hooks calling ``torch.distributed._functional_collectives.all_reduce``) run under a gloo process group of
2 and 4 CPU ranks on tiny Llama (GQA) and Mixtral configs.

Run once here (never on the GPU box; /root/reference does not exist there):
    python tests/golden/make_golden_tp.py
Writes ``g4_tp_logits.npz``: per (family, world, weights, dtype) the logits of a 12-token prefill and 8 greedy
decode steps (teacher-forced on the reference's own greedy tokens, identical on every rank), the tokens, and the
prompt; for every bf16 run also ``{key}_logits_f32``: the same weights in fp32, teacher-forced on the bf16 run's
tokens (the exact-arithmetic side of the GPU tests' accuracy bound, tests/parity.py). Weights come from ``oracle.synth`` (regenerable anywhere). ``weights = "q4g"``: after sharding, every
Linear (lm_head included, unsharded) holds dequant(quant_int4(shard)) with the product's group rule (128, or the
largest of 64 / 32 dividing the shard's in_features) — the order of the reference's BitsandbytesPrecision
convert -> tensor_parallel -> quantize-on-device (generate/tp.py:171-190).
"""

from __future__ import annotations

import os
import sys
import tempfile
from pathlib import Path
from unittest.mock import Mock

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(HERE))

FAMILIES = {
    # head_size 64 (n_embd 512 / 8 heads): a head size the MI355X attention kernels run, so the product's TP decode
    # can be compared with these logits on the GPU
    "llama": ("Llama-2-70b-hf", dict(n_layer=2, n_embd=512, n_head=8, n_query_groups=4, intermediate_size=1024,
                                     vocab_size=1000, padding_multiple=64, block_size=64)),
    "mixtral": ("Mixtral-8x7B-v0.1", dict(n_layer=2, n_embd=512, n_head=8, n_query_groups=4, intermediate_size=1024,
                                          n_expert=4, n_expert_per_token=2, padded_vocab_size=1024, vocab_size=1024,
                                          block_size=64)),
    # GPT-NeoX (pythia): biased Linears (the row-parallel proj bias stays whole on every rank, generate/tp.py:43-45),
    # LayerNorm, partial rotary (16 of 64 dims), parallel residual, GELU MLP
    "neox": ("pythia-160m", dict(n_layer=2, n_embd=512, n_head=8, intermediate_size=1024, vocab_size=1000,
                                 padded_vocab_size=1024, block_size=64)),
}
VARIANTS = [("fp32", torch.float32), ("fp32", torch.bfloat16), ("q4g", torch.bfloat16)]
T, STEPS = 12, 8


def fit_group(K, group=128):
    for g in (group, 128, 64, 32):
        if g <= group and K % g == 0:
            return g
    raise ValueError(K)


def q4g_shards(model):
    from oracle import quant

    for mod in model.modules():
        if isinstance(mod, torch.nn.Linear):
            w = mod.weight.detach().float().numpy()
            g = fit_group(w.shape[1])
            mod.weight.data = torch.from_numpy(quant.dequantize_q4g(*quant.quantize_q4g(w, g), g))


def worker(rank, world, tmp, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import make_golden
    from oracle import synth

    config, model_mod, gbase, gtp = make_golden.import_reference()
    out = {}
    for fam, (name, kw) in FAMILIES.items():
        cfg = config.Config.from_name(name, **kw)
        sd = synth.state_dict(cfg, seed=17)
        prompt = torch.from_numpy(synth.token_ids(T, cfg.vocab_size, seed=17)).long()
        for wname, dtype in VARIANTS:
            def build(dt):
                m = model_mod.GPT(config.Config.from_name(name, **kw))  # tensor_parallel divides the config in place
                m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
                fab = Mock()
                fab.world_size, fab.global_rank = world, rank
                gtp.tensor_parallel(fab, m)
                if wname == "q4g":
                    q4g_shards(m)
                m = m.to(dt).eval()
                m.max_seq_length = T + STEPS + 1
                m.set_kv_cache(batch_size=1)
                return m

            def run(m, forced=None):
                with torch.inference_mode():
                    lg = m(prompt.view(1, -1), torch.arange(T))[0, -1].float()
                    logits, toks = [lg], [int(torch.argmax(lg))]
                    for s in range(STEPS):
                        tok = toks[-1] if forced is None else int(forced[s])
                        lg = m(torch.tensor([[tok]]), torch.tensor([T + s]))[0, -1].float()
                        logits.append(lg)
                        toks.append(int(torch.argmax(lg)))
                return torch.stack(logits).numpy(), np.array(toks, dtype=np.int64)

            key = f"{fam}_w{world}_{wname}_{str(dtype).split('.')[-1]}"
            out[f"{key}_logits"], out[f"{key}_tokens"] = run(build(dtype))
            if dtype == torch.bfloat16:
                out[f"{key}_logits_f32"], _ = run(build(torch.float32), forced=out[f"{key}_tokens"])
        out[f"{fam}_prompt"] = prompt.numpy()
    if rank == 0:
        np.savez(Path(tmp) / f"w{world}.npz", **out)
    dist.barrier()
    dist.destroy_process_group()


def main():
    import socket

    merged = {}
    with tempfile.TemporaryDirectory() as tmp:
        for world in (2, 4):
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            mp.spawn(worker, args=(world, tmp, port), nprocs=world, join=True)
            merged.update(dict(np.load(Path(tmp) / f"w{world}.npz")))
    np.savez_compressed(HERE / "g4_tp_logits.npz", **merged)
    print("wrote", sorted(k for k in merged if k.endswith("_tokens")))


if __name__ == "__main__":
    main()
