"""The TP all-reduce's push phase timed in ONE process on one GPU (VERDICT r5 "Next round" item 6).

usage: python tools/ar_push_time.py [--calls 64]

Rank 0 of an 8-rank world runs alone: all eight mailboxes are local allocations (lga_comm_alloc), and the seven peer
flags in rank 0's own mailbox are pre-set past every sequence number the run reaches, so the flag wait passes at once
and nothing waits on another process. Per call the protocol records (lga_comm_trace) give entry -> flags raised (the
push: 7 x n bf16 written system-coherent into the peers' mailboxes, drained, plus the flag stores; for the fused
GEMV form the record starts at the rank's last-arriving workgroup, after every workgroup pushed its rows) and raised -> wait
done; HIP events over back-to-back launches give the whole call. Measured for lga_allreduce_bf16 at the 7B / 70B
hidden sizes and for the fused row-parallel GEMV + all-reduce (lga_q4_gemv_allreduce) at the 7B TP = 8 rank's
attn.proj (K = 512) and mlp.proj (K = 1376, group 32) and the 70B TP = 8 rank's (K = 1024 / 3584).
This is the push into LOCAL uncached HBM: the cross-GPU term adds the xGMI store latency on top.
"""

import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]

from lit_gpt import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=64)
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.zeros(1, device=dev)
    lib = ops.load_library()
    hip = ctypes.CDLL("libamdhip64.so")
    world, cap = 8, 16384
    mb_bytes = lib.lga_comm_mailbox_bytes(cap)
    mbs = []
    for _ in range(world):
        ptr, handle = ctypes.c_void_p(), ctypes.create_string_buffer(64)
        ops._check(lib.lga_comm_alloc(mb_bytes, ctypes.byref(ptr), handle))
        mbs.append(ptr.value)
    # rank 0's own mailbox: flags[8] (uint32, 256 B apart); peers 1..7 pre-set far ahead of any sequence number
    flags = np.zeros(8 * 64, dtype=np.uint32)
    for r in range(1, world):
        flags[r * 64] = 0x7FFFFFFF
    rc = hip.hipMemcpy(ctypes.c_void_p(mbs[0]), flags.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(flags.nbytes), 1)
    assert rc == 0, rc
    # the tagged protocol's granules from peers 1..7 in rank 0's own mailbox (both slots), tags far ahead as well
    gran_off = 8 * 64 * 4 + 2 * 8 * cap * 2
    gran = np.zeros((2, 8, cap // 2, 2), dtype=np.uint32)
    gran[:, 1:, :, 1] = 0x7FFFFFFF
    rc = hip.hipMemcpy(ctypes.c_void_p(mbs[0] + gran_off), gran.ctypes.data_as(ctypes.c_void_p),
                       ctypes.c_size_t(gran.nbytes), 1)
    assert rc == 0, rc
    tagged = hasattr(lib, "lga_q4_gemv_allreduce_tagged")
    torch.cuda.synchronize()
    mb_arr = (ctypes.c_void_p * world)(*mbs)
    seq = torch.zeros(1, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    arrive = torch.zeros(640, dtype=torch.int32, device=dev)
    n_rec = 4 * args.calls + 16
    trace = torch.zeros(n_rec, 16, dtype=torch.int64, device=dev)
    ops._check(lib.lga_comm_trace(ctypes.c_void_p(trace.data_ptr()), n_rec))
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731

    def measure(name, call):
        trace.zero_()
        seq.zero_()
        call()  # warm (also builds the kernel)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()  # back-to-back launches without host gaps
        with torch.cuda.graph(g):
            for _ in range(args.calls):
                call()
        torch.cuda.synchronize()
        trace.zero_()
        seq.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert int(err.item()) == 0, "flag wait timed out"
        tr = trace.cpu().numpy().astype(np.int64)[: args.calls]
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        push = (tr[:, 2] - tr[:, 1]) / 100.0  # 100 MHz clock -> us
        wait = (tr[:, 3] - tr[:, 2]) / 100.0
        per = s.elapsed_time(e) * 1e3 / args.calls
        what = "last arrival -> raised" if "gemv" in name else "entry -> raised"
        print(f"{name:44s} call {per:6.2f} us | {what} median {np.median(push):5.2f} us "
              f"(p10 {np.percentile(push, 10):5.2f}, p90 {np.percentile(push, 90):5.2f}, max {push.max():5.2f}) | "
              f"raised -> wait done {np.median(wait):5.2f}", flush=True)

    for n in (4096, 8192):
        x = torch.randn(n, device=dev).bfloat16()
        res = torch.randn(n, device=dev).bfloat16()
        y = torch.empty_like(x)
        measure(f"lga_allreduce_bf16 n={n}", lambda: ops._check(lib.lga_allreduce_bf16(
            ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(res.data_ptr()), ctypes.c_void_p(y.data_ptr()), n, mb_arr,
            0, world, cap, ctypes.c_void_p(seq.data_ptr()), ctypes.c_void_p(err.data_ptr()), st())))
    from lit_gpt.quantize import _fit_group

    for label, N, K in (("7B tp8 attn.proj", 4096, 512), ("7B tp8 mlp.proj", 4096, 1376),
                        ("70B tp8 attn.proj", 8192, 1024), ("70B tp8 mlp.proj", 8192, 3584)):
        g = _fit_group(K, 128)
        qw, sc = ops.quantize(torch.randn(N, K, device=dev) * 0.02, ops.FMT_Q4G, g)
        x = torch.randn(K, device=dev).bfloat16()
        res = torch.randn(N, device=dev).bfloat16()
        y = torch.empty(N, device=dev, dtype=torch.bfloat16)
        measure(f"lga_q4_gemv_allreduce {label} N={N} K={K}", lambda: ops._check(lib.lga_q4_gemv_allreduce(
            ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(qw.data_ptr()), ctypes.c_void_p(sc.data_ptr()), None,
            ctypes.c_void_p(res.data_ptr()), ctypes.c_void_p(y.data_ptr()), N, K, g, 0, mb_arr, 0, world, cap,
            ctypes.c_void_p(seq.data_ptr()), ctypes.c_void_p(arrive.data_ptr()), ctypes.c_void_p(err.data_ptr()),
            st())))
        if tagged:
            measure(f"lga_q4_gemv_allreduce_tagged {label}", lambda: ops._check(lib.lga_q4_gemv_allreduce_tagged(
                ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(qw.data_ptr()), ctypes.c_void_p(sc.data_ptr()), None,
                ctypes.c_void_p(res.data_ptr()), ctypes.c_void_p(y.data_ptr()), N, K, g, 0, mb_arr, 0, world, cap,
                ctypes.c_void_p(seq.data_ptr()), ctypes.c_void_p(arrive.data_ptr()), ctypes.c_void_p(err.data_ptr()),
                st())))
        # the same GEMV alone (no all-reduce) for the difference
        ops.q4_gemv(x, qw, sc, N, K, g, 0, residual=res, out=y)
        torch.cuda.synchronize()
        gg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gg):
            for _ in range(args.calls):
                ops.q4_gemv(x, qw, sc, N, K, g, 0, residual=res, out=y)
        gg.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        gg.replay()
        e.record()
        e.synchronize()
        print(f"{'  lga_q4_gemv alone (same shape)':44s} call {s.elapsed_time(e) * 1e3 / args.calls:6.2f} us", flush=True)
    ops._check(lib.lga_comm_trace(None, 0))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
