"""Worker for tests/test_gpu_tp.py::test_fused_gemv_allreduce_* (torch.distributed.run, every rank on cuda:0, gloo
group for the IPC-handle exchange). Each rank holds a row-parallel 4-bit shard (the attn.proj / mlp.proj split of
generate/tp.py) and runs ``XgmiAllReduce.gemv_all_reduce`` — the GEMV with the all-reduce in its epilogue,
lga_q4_gemv_allreduce — against the two-launch form it replaces (lga_q4_gemv, then lga_allreduce_bf16): results
must be bit-identical, eagerly, from a captured HIP graph replayed with new inputs, interleaved with plain
all-reduce calls (one shared call sequence), and back to back without host synchronisation. Writes a status file."""

import os
import sys
from pathlib import Path

import torch
import torch.distributed as dist

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO), str(Path(__file__).resolve().parent)]

from lit_gpt import comm  # noqa: E402
from lit_gpt.quantize import QuantLinear  # noqa: E402

DEV = torch.device("cuda", 0)


def rnd(shape, seed, scale=1.0):
    return (torch.randn(*shape, generator=torch.Generator().manual_seed(seed)) * scale)


@torch.inference_mode()
def main():
    out = sys.argv[1]
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    c = comm.XgmiAllReduce(device=DEV)
    if "--late-peer" in sys.argv:
        return late_peer(c, out, world, rank)
    if "--time" in sys.argv:
        return timing(c, out, world, rank)
    bad = [] if c.fused_ok else [f"start-up self-test: {c.fused_fallback}"]
    want = os.environ.get("LGA_AR_PROTOCOL")
    if want in ("flags", "tagged") and c.protocol != want:
        bad.append(f"protocol {c.protocol}, asked for {want}")
    if bad:  # a broken protocol would make every later call wait out its 5 s bound: report and stop here
        dist.barrier()
        c.close()
        if rank == 0:
            Path(out).write_text(f"FAIL {bad}")
            Path(out + ".trace.txt").write_text("")
        dist.destroy_process_group()
        return
    c.enable_trace(512)  # every call's protocol record, per rank (allreduce_worker.trace_report)
    # (N, K per rank, mode, bias): 7B attn.proj / mlp.proj shards at this world size, 70B-like widths, fp4 / nf4
    cases = [(4096, 4096 // world, "int4-g128", False), (4096, 11008 // world, "int4-g128", False),
             (8192, 8192 // world, "nf4", False), (4096, 2048, "bnb.fp4", True), (1024, 1376, "int4-g32", False)]
    for ci, (N, K, mode, use_bias) in enumerate(cases):
        w = rnd((N, K), 100 * ci + rank, 0.02).bfloat16().to(DEV)
        b = rnd((N,), 7 + ci, 0.1).bfloat16().to(DEV) if use_bias else None
        lin = QuantLinear.from_float(w, b, mode, DEV)
        for it in range(3):
            x = rnd((K,), 1000 * ci + 10 * it + rank).bfloat16().to(DEV)
            res = rnd((N,), 5000 + it, 2.0).bfloat16().to(DEV) if it != 1 else None
            fused = c.gemv_all_reduce(lin, x, res)
            two = c.all_reduce(lin(x.view(1, -1)).view(-1), residual=res)
            if not torch.equal(fused, two):
                bad.append(f"eager case {ci} ({N}x{K} {mode}) it {it}: max diff "
                           f"{(fused.float() - two.float()).abs().max().item()}")
    # graph: fused calls interleaved with plain all-reduces on static buffers, new inputs between replays
    N, K = 4096, 11008 // world
    lin = QuantLinear.from_float(rnd((N, K), 77 + rank, 0.02).bfloat16().to(DEV), None, "int4-g128", DEV)
    xs = torch.empty(K, dtype=torch.bfloat16, device=DEV)
    res = torch.empty(N, dtype=torch.bfloat16, device=DEV)
    ya, yb, yc = (torch.empty(N, dtype=torch.bfloat16, device=DEV) for _ in range(3))
    torch.cuda.synchronize()
    dist.barrier()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        c.gemv_all_reduce(lin, xs, res, out=ya)
        c.all_reduce(ya, out=yb)  # a plain call in the same sequence
        c.gemv_all_reduce(lin, xs, None, out=yc)
    for rep in range(4):
        xs.copy_(rnd((K,), 9000 + 10 * rep + rank).bfloat16())
        res.copy_(rnd((N,), 9500 + rep).bfloat16())
        torch.cuda.synchronize()
        dist.barrier()
        g.replay()
        torch.cuda.synchronize()
        part = lin(xs.view(1, -1)).view(-1)
        ea = c.all_reduce(part, residual=res)
        eb = c.all_reduce(ea)
        ec = c.all_reduce(part)
        torch.cuda.synchronize()
        for name, got, exp in (("a", ya, ea), ("b", yb, eb), ("c", yc, ec)):
            if not torch.equal(got, exp):
                bad.append(f"graph replay {rep} output {name}")
    # back to back, no host synchronisation (ranks drift; the two mailbox slots keep them apart)
    outs, exps = [], []
    for k in range(48):
        x = rnd((K,), 20000 + 10 * k + rank).bfloat16().to(DEV)
        outs.append(c.gemv_all_reduce(lin, x))
        exps.append(lin(x.view(1, -1)).view(-1))
    refs = [c.all_reduce(e) for e in exps]
    torch.cuda.synchronize()
    for k, (y, r) in enumerate(zip(outs, refs)):
        if not torch.equal(y, r):
            bad.append(f"burst call {k}")
            break
    err = c.errors()
    from allreduce_worker import trace_report

    report = trace_report(c, world, rank, bad, err)
    dist.barrier()
    c.close()
    if rank == 0:
        Path(out + ".trace.txt").write_text(report)
        Path(out).write_text("ok" if not bad and err == 0 else f"FAIL err={err} {bad[:5]}\n{report[-6000:]}")
    dist.destroy_process_group()


def timing(c, out, world, rank):
    """us per call, graph-captured (32 calls per replay), of the fused launch vs GEMV + all-reduce for the 7B
    attn.proj / mlp.proj shards at this world size — every rank on one GPU, so both forms share the device: a
    relative number, not a multi-GPU one (tools/tp_fused_time.py)."""
    res_lines = []
    for name, N, K in (("attn.proj", 4096, 4096 // world), ("mlp.proj", 4096, 11008 // world)):
        lin = QuantLinear.from_float(rnd((N, K), 5 + rank, 0.02).bfloat16().to(DEV), None, "int4-g128", DEV)
        x = rnd((K,), 11 + rank).bfloat16().to(DEV)
        res = rnd((N,), 12).bfloat16().to(DEV)
        ys = [torch.empty(N, dtype=torch.bfloat16, device=DEV) for _ in range(2)]
        part = torch.empty(1, N, dtype=torch.bfloat16, device=DEV)
        times = {}
        for form in ("fused", "two"):
            def call():
                if form == "fused":
                    c.gemv_all_reduce(lin, x, res, out=ys[0])
                else:
                    from lit_gpt import ops
                    ops.q4_gemv(x, lin.qweight, lin.scales, N, K, lin.group, lin.fmt, out=part.view(-1))
                    c.all_reduce(part.view(-1), residual=res, out=ys[1])
            for _ in range(4):
                call()
            torch.cuda.synchronize()
            dist.barrier()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(32):
                    call()
            best = 1e9
            for _ in range(5):
                torch.cuda.synchronize()
                dist.barrier()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                g.replay()
                e.record()
                e.synchronize()
                best = min(best, s.elapsed_time(e) * 1e3 / 32)
            times[form] = best
        res_lines.append(f"world {world} {name} N={N} K={K}: fused {times['fused']:.2f} us, "
                         f"gemv + all-reduce {times['two']:.2f} us per call (rank {rank})")
    dist.barrier()
    c.close()
    if rank == 0:
        Path(out).write_text("\n".join(res_lines) + "\n")
    dist.destroy_process_group()


def late_peer(c, out, world, rank):
    """The last rank reaches the fused call 6 s after the others: the early ranks' last-arriving workgroups give up
    after 5 s and set the error word (no GPU hang); comm.check_errors raises AllReduceTimeout on every rank."""
    import time

    lin = QuantLinear.from_float(rnd((4096, 512), rank, 0.02).bfloat16().to(DEV), None, "int4-g128", DEV)
    x = rnd((512,), 3 + rank).bfloat16().to(DEV)
    torch.cuda.synchronize()
    dist.barrier()
    if rank == world - 1:
        time.sleep(6.0)
    c.gemv_all_reduce(lin, x)
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
