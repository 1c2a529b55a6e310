"""Worker for the tensor-parallel parity tests (tests/test_gpu_tp.py), launched by torch.distributed.run.

All ranks share cuda:0 (the box has one GPU); the process group is gloo (RCCL refuses two ranks on one device).
Every rank builds its shard with the product entry point ``generate.base.build_model(fabric=...)`` (per-block
sharding of generate/tp.py + per-shard quantization), runs ``--steps`` tokens (a prefill of ``--T`` prompt ids, or
with ``--cache P`` a synthetic KV context of P positions written into every rank's cache slice, then decode steps)
and keeps its logits. The decode all-reduces use the xGMI one-shot kernel (lit_gpt/comm.py) with ``--allreduce
xgmi`` — several ranks' kernels then wait on each other on the same device — or gloo.

Rank 0 then assembles the UNSHARDED weights from every rank's packed shard (colwise shards concatenated along
dim 0, rowwise along dim 1, replicated tensors from rank 0), dequantizes them with oracle/quant.py, runs the
oracle (CPU restatement of the reference) teacher-forced on the same tokens, and writes per-step logits of both
plus the router gaps (MoE) to ``out``.
"""

import argparse
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]

from generate import tp as gtp  # noqa: E402
from generate.base import build_model  # noqa: E402
from lit_gpt import Config, comm  # noqa: E402
from lit_gpt.quantize import QuantLinear  # noqa: E402
from oracle import model as om  # noqa: E402
from oracle import quant, synth  # noqa: E402

DEV = torch.device("cuda", 0)
COLWISE = (".attn.attn", ".fc_1", ".fc_2", ".mlp.fc")
ROWWISE = (".attn.proj", ".mlp.proj", ".proj")


def style(name: str):
    if any(name.endswith(s) for s in COLWISE):
        return 0
    if any(name.endswith(s) for s in ROWWISE) and name != "lm_head":
        return 1
    return None


def shard_state(model):
    """name -> (array, kind) with kind 'q4g:<group>' / 'nf4:<group>' (packed, scales) or 'dense'."""
    out = {}
    for name, mod in model.named_modules():
        if isinstance(mod, QuantLinear):
            sc = mod.scales.view(torch.int16).cpu().numpy().view(np.uint16) if mod.fmt == 0 else mod.scales.cpu().numpy()
            out[f"{name}.weight"] = ("q4g" if mod.fmt == 0 else "nf4", mod.group, mod.qweight.cpu().numpy(), sc)
            if mod.bias is not None:
                out[f"{name}.bias"] = ("dense", 0, mod.bias.float().cpu().numpy(), None)
    for name, p in model.named_parameters():
        if name not in out:
            out[name] = ("dense", 0, p.detach().float().cpu().numpy(), None)
    return out


def dequant(entry):
    kind, group, a, sc = entry
    if kind == "q4g":
        return quant.dequantize_q4g(a, sc, group)
    if kind == "nf4":
        return quant.dequantize_nf4(a, sc, group)
    return a


def synthetic_cache(cfg, P):
    """Full-model K/V context (G, P, hs) per layer, bf16-representable, seeded."""
    rng = np.random.default_rng(2024)
    out = []
    for _ in range(cfg.n_layer):
        k = rng.standard_normal((cfg.n_query_groups, P, cfg.head_size), dtype=np.float32)
        v = rng.standard_normal((cfg.n_query_groups, P, cfg.head_size), dtype=np.float32)
        out.append((torch.from_numpy(k).bfloat16(), torch.from_numpy(v).bfloat16()))
    return out


def router_gap_hooks(model, gaps):
    for blk in model.transformer.h:
        if hasattr(blk.mlp, "gate"):
            k = model.config.n_expert_per_token

            def hook(m, a, o, k=k):
                v = torch.sort(o.float().reshape(-1, o.size(-1)), dim=-1, descending=True).values
                gaps.append(float((v[:, k - 1] - v[:, k]).min()))

            blk.mlp.gate.register_forward_hook(hook)


@torch.inference_mode()
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--model", default="Llama-2-70b-hf")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--mode", default="int4-g128")
    ap.add_argument("--T", type=int, default=16)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--cache", type=int, default=0, help="synthetic KV context length instead of a prompt")
    ap.add_argument("--allreduce", default="xgmi", choices=["xgmi", "gloo"])
    ap.add_argument("--graph", action="store_true", help="also run greedy decode through the HIP graph")
    ap.add_argument("--greedy", action="store_true", help="feed each step the previous argmax (eager generate)")
    ap.add_argument("--sampled", action="store_true",
                    help="also run generate(temperature=0.8, top_k=200) after torch.manual_seed(1234) on every rank")
    ap.add_argument("--tmp", required=True)
    args = ap.parse_args()
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    if args.allreduce == "xgmi":
        comm.set_default(comm.XgmiAllReduce(device=DEV))
    cfg = Config.from_name(args.model, n_layer=args.layers)
    full_cfg = Config.from_name(args.model, n_layer=args.layers)
    fabric = gtp.Fabric(world, rank)
    P = args.cache
    max_seq = (P if P else args.T) + args.steps + 1
    model = build_model(cfg, quantize=None if args.mode == "bf16" else args.mode, device=DEV, seed=3,
                        max_seq_length=max_seq, fabric=fabric)
    gaps = []
    router_gap_hooks(model, gaps)
    ids = torch.from_numpy(synth.token_ids(args.T + args.steps, full_cfg.vocab_size, seed=9)).to(torch.int32)
    cache = None
    if P:
        cache = synthetic_cache(full_cfg, P)
        Gr = cfg.n_query_groups  # groups of this rank
        for i, blk in enumerate(model.transformer.h):
            k, v = cache[i]
            blk.attn.kv_cache.k[0, :, :P] = k[rank * Gr:(rank + 1) * Gr].to(DEV)
            blk.attn.kv_cache.v[0, :, :P] = v[rank * Gr:(rank + 1) * Gr].to(DEV)
    logits, step_gaps, fed = [], [], []

    def record(lg):
        logits.append(lg[0, -1].float().cpu())
        step_gaps.append(min(gaps, default=float("inf")))
        gaps.clear()

    def next_id(s):  # teacher-forced synthetic ids, or (--greedy) the argmax of the previous step
        return int(torch.argmax(logits[-1])) if args.greedy else int(ids[(0 if P else args.T) + s])

    T = args.T
    if not P:
        record(model(ids[:T].view(1, -1).to(DEV), torch.arange(T, device=DEV), last_token_only=True))
    base = P if P else T
    for s in range(args.steps if P else args.steps - 1):
        tok = next_id(s)
        fed.append(tok)
        record(model(torch.tensor([[tok]], device=DEV), torch.tensor([base + s], device=DEV), last_token_only=True))
    graph_tokens = np.zeros(0, dtype=np.int32)
    if args.graph and not P:
        from generate.base import generate

        for b in model.transformer.h:
            b.attn.kv_cache.reset_parameters()
        y = generate(model, ids[:T].to(DEV), T + args.steps, temperature=0.0)
        graph_tokens = y[T:].cpu().numpy()
    sampled_tokens = np.zeros(0, dtype=np.int64)
    if args.sampled and not P:
        from generate.base import generate

        for b in model.transformer.h:
            b.attn.kv_cache.reset_parameters()
        torch.manual_seed(1234)  # every rank draws the same sampler seed from its generator (replicated sampling)
        y = generate(model, ids[:T].to(DEV), T + args.steps, temperature=0.8, top_k=200)
        sampled_tokens = y[T:].cpu().numpy().astype(np.int64)
    sl = [None] * world
    dist.all_gather_object(sl, sampled_tokens)
    sampled_same = all(np.array_equal(sl[0], t) for t in sl)
    err = comm.get_default().errors() if comm.get_default() is not None else 0
    torch.cuda.synchronize()
    tmp = Path(args.tmp)
    st = shard_state(model)
    np.savez(tmp / f"rank{rank}.npz", **{f"{k}|{e[0]}|{e[1]}|a": e[2] for k, e in st.items()},
             **{f"{k}|{e[0]}|{e[1]}|s": e[3] for k, e in st.items() if e[3] is not None})
    got = torch.stack(logits).numpy()
    # every rank must hold bit-identical logits (replicated sampling, generate/tp.py)
    gl = [None] * world
    dist.all_gather_object(gl, got)
    same_across_ranks = all(np.array_equal(gl[0], g) for g in gl)
    dist.barrier()
    del model
    torch.cuda.empty_cache()
    if rank == 0:
        t0 = time.time()
        parts = [np.load(tmp / f"rank{r}.npz") for r in range(world)]
        names = sorted({k.split("|")[0] for k in parts[0].files})
        sd = {}
        for name in names:
            key = next(k for k in parts[0].files if k.startswith(name + "|") and k.endswith("|a"))
            _, kind, group, _ = key.split("|")
            entries = []
            for p in parts:
                a = p[key]
                s = p[key[:-2] + "|s"] if kind != "dense" else None
                entries.append(dequant((kind, int(group), a, s)))
            st_ = style(name.rsplit(".", 1)[0]) if name.endswith(".weight") else (
                0 if style(name.rsplit(".", 1)[0]) == 0 else None)
            sd[name] = np.concatenate(entries, axis=st_) if st_ is not None and world > 1 else entries[0]
        def run_oracle(dtype):
            ref = om.OracleGPT(full_cfg, sd, dtype=dtype, rope_pos_dtype=torch.bfloat16)
            ref.set_kv_cache(max_seq)
            rgaps = []
            orig = ref._lin

            def lin(name, x, *a, **kw):
                y = orig(name, x, *a, **kw)
                if name.endswith("mlp.gate"):
                    v = torch.sort(y.float(), dim=-1, descending=True).values
                    k = full_cfg.n_expert_per_token
                    rgaps.append(float((v[:, k - 1] - v[:, k]).min()))
                return y

            ref._lin = lin
            exp, ref_step_gaps = [], []

            def ref_record(lg):
                exp.append(lg[-1].double())
                ref_step_gaps.append(min(rgaps, default=float("inf")))
                rgaps.clear()

            if P:
                for i in range(full_cfg.n_layer):
                    ref.cache.write(i, torch.arange(P), cache[i][0].to(dtype), cache[i][1].to(dtype))
            else:
                ref_record(ref.forward(ids[:T].long(), torch.arange(T), last_only=True))
            for s, tok in enumerate(fed):
                ref_record(ref.forward(torch.tensor([tok]), torch.tensor([base + s])))
            return torch.stack(exp).numpy(), ref_step_gaps

        exp, ref_step_gaps = run_oracle(torch.bfloat16)
        exp64, gaps64 = run_oracle(torch.float64)  # exact-arithmetic side of tests/parity.py
        ref_step_gaps = np.minimum(ref_step_gaps, gaps64)
        np.savez(args.out, tp=got, ref=exp, ref64=exp64, gaps=np.array(step_gaps),
                 ref_gaps=np.array(ref_step_gaps), same_across_ranks=same_across_ranks,
                 comm_err=err, graph_tokens=graph_tokens, fed=np.array(fed), oracle_s=time.time() - t0,
                 sampled_tokens=sampled_tokens, sampled_same=sampled_same)
    dist.barrier()
    if comm.get_default() is not None:
        comm.get_default().close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
