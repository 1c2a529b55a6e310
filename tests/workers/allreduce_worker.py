"""Worker for tests/test_gpu_tp.py::test_xgmi_allreduce_* (launched by torch.distributed.run; all ranks on cuda:0,
gloo group for the IPC-handle exchange). Every rank reduces seeded partials through lga_allreduce_bf16 — eagerly and
from a captured HIP graph replayed several times — and checks each result bit-exactly against the ordered fp32
sum over ranks 0..W-1 rounded once to bf16 (plus the residual add in the Block's rounding). Writes a status file."""

import os
import sys
from pathlib import Path

import torch
import torch.distributed as dist

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]

from lit_gpt import comm  # noqa: E402

DEV = torch.device("cuda", 0)


def partial(rank, n, it):
    g = torch.Generator().manual_seed(1000 * it + rank)
    return (torch.randn(n, generator=g) * (1 + rank)).bfloat16()


def expected(world, n, it, residual=None):
    acc = torch.zeros(n, dtype=torch.float32)
    for r in range(world):
        acc += partial(r, n, it).float()
    y = acc.bfloat16()
    return y if residual is None else (y.float() + residual.float()).bfloat16()


@torch.inference_mode()
def main():
    out = sys.argv[1]
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    c = comm.XgmiAllReduce(device=DEV)
    if "--late-peer" in sys.argv:
        return late_peer(c, out, world, rank)
    c.enable_trace(512)  # every call's protocol record (entry / flags raised / wait done / flags seen), per rank
    bad = []
    it = 0
    for n in (4096, 8192, 32768, 8):
        for use_res in (False, True):
            it += 1
            x = partial(rank, n, it).to(DEV)
            res = (torch.randn(n, generator=torch.Generator().manual_seed(it)) * 3).bfloat16()
            y = c.all_reduce(x, residual=res.to(DEV) if use_res else None).cpu()
            if not torch.equal(y, expected(world, n, it, res if use_res else None)):
                bad.append(f"eager n={n} res={use_res}")
    # graph capture: 3 calls per replay on static buffers, new data written between replays
    n = 4096
    xs = [torch.empty(n, dtype=torch.bfloat16, device=DEV) for _ in range(3)]
    ys = [torch.empty(n, dtype=torch.bfloat16, device=DEV) for _ in range(3)]
    res = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    for i in range(3):
        xs[i].copy_(partial(rank, n, 100 + i))
    res.copy_(torch.ones(n).bfloat16())
    torch.cuda.synchronize()
    dist.barrier()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(3):
            c.all_reduce(xs[i], residual=res if i == 1 else None, out=ys[i])
    for rep in range(5):
        its = [200 + 10 * rep + i for i in range(3)]
        for i in range(3):
            xs[i].copy_(partial(rank, n, its[i]))
        torch.cuda.synchronize()
        dist.barrier()
        g.replay()
        torch.cuda.synchronize()
        for i in range(3):
            exp = expected(world, n, its[i], torch.ones(n).bfloat16() if i == 1 else None)
            if not torch.equal(ys[i].cpu(), exp):
                bad.append(f"graph replay {rep} call {i}")
    # back-to-back eager calls without host synchronisation (ranks drift; the two mailbox slots keep them apart)
    outs = []
    for k in range(64):
        outs.append(c.all_reduce(partial(rank, 1024, 500 + k).to(DEV)))
    torch.cuda.synchronize()
    for k, y in enumerate(outs):
        if not torch.equal(y.cpu(), expected(world, 1024, 500 + k)):
            bad.append(f"burst call {k}")
            break
    err = c.errors()
    report = trace_report(c, world, rank, bad, err)
    dist.barrier()
    c.close()
    if rank == 0:
        Path(out + ".trace.txt").write_text(report)
        Path(out).write_text("ok" if not bad and err == 0 else f"FAIL err={err} {bad[:5]}\n{report[-6000:]}")
    dist.destroy_process_group()


def trace_report(c, world, rank, bad, err):
    """Every rank's protocol records, gathered on rank 0: per call (sequence number) and rank the entry, flags-raised
    and wait-done times (us from the earliest entry of that call on any rank; one clock per device), whether the wait
    timed out, the sequence word read at entry and the flag words seen. Failing or slow calls are listed in full."""
    import numpy as np

    mine = {"rank": rank, "trace": c.traces(), "seq": int(c.seq.item()), "err": int(err), "bad": bad}
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    if rank != 0:
        return ""
    lines = [f"ranks {world}; per rank: seq counter " + " ".join(str(d["seq"]) for d in allr)
             + "; err " + " ".join(str(d["err"]) for d in allr)]
    seqs = sorted({int(r[0]) & 0xFFFFFFFF for d in allr for r in d["trace"] if r[0]})
    worst = []
    for s in seqs:
        recs = []
        for d in allr:
            r = [x for x in d["trace"] if x[0] and (int(x[0]) & 0xFFFFFFFF) == s]
            recs.append(r[0] if r else None)
        if any(x is None for x in recs):
            worst.append((1e9, s, recs))
            continue
        t0 = min(int(x[1]) for x in recs)
        span = (max(int(x[3]) for x in recs) - t0) / 100.0
        worst.append((span + (1e8 if any(int(x[4]) for x in recs) else 0), s, recs))
    worst.sort(key=lambda w: -w[0])
    spans = sorted(w[0] for w in worst if w[0] < 1e8)
    if spans:
        lines.append(f"calls {len(seqs)}; entry->last wait done us: median {np.median(spans):.1f} "
                     f"p90 {np.percentile(spans, 90):.1f} max {spans[-1]:.1f}")
    for score, s, recs in worst[:6]:
        lines.append(f"seq {s}:" + (" TIMED OUT" if score >= 1e8 else "") + ("" if score < 1e9 else " (missing)"))
        ok = [x for x in recs if x is not None]
        t0 = min(int(x[1]) for x in ok) if ok else 0
        for r, x in enumerate(recs):
            if x is None:
                lines.append(f"   rank {r}: no record")
                continue
            kind = {1: "oneshot", 2: "gemv"}.get(int(x[0]) >> 40, "?")
            lines.append(f"   rank {r} {kind}: entry {(int(x[1]) - t0) / 100:9.2f} raised {(int(x[2]) - t0) / 100:9.2f} "
                         f"done {(int(x[3]) - t0) / 100:9.2f} timeout {int(x[4])} seqword {int(x[5])} "
                         f"flags {[int(v) for v in x[6:6 + world]]}")
    return "\n".join(lines) + "\n"


def late_peer(c, out, world, rank):
    """The last rank reaches the all-reduce 6 s after the others (past the kernel's 5 s peer bound): the early
    ranks' kernels give up and set the error word; comm.check_errors must then raise AllReduceTimeout on EVERY
    rank, the late one included (a lost peer must not yield silent partial sums)."""
    import time

    x = partial(rank, 4096, 1).to(DEV)
    torch.cuda.synchronize()
    dist.barrier()
    if rank == world - 1:
        time.sleep(6.0)
    c.all_reduce(x)
    torch.cuda.synchronize()
    raised = 0
    try:
        comm.check_errors(c)
    except comm.AllReduceTimeout:
        raised = 1
    flags = [None] * world
    dist.all_gather_object(flags, raised)
    dist.barrier()
    c.close()
    if rank == 0:
        Path(out).write_text("ok" if all(flags) else f"FAIL raised per rank: {flags}")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
