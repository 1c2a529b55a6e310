"""Lab probe: does streaming the NEXT kernel's weights through the Infinity Cache (MALL) on a side stream shorten
the decode GEMV chain?  Uses the fc_1||fc_2 SwiGLU GEMV shape of Llama-2-7B (46.5 MB per launch).

usage: python tools/mall_probe.py     (needs tools/_lab/prefetch_lab.so, see tools/prefetch_lab.hip)
"""
import ctypes
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
from lit_gpt import ops  # noqa: E402

lab = ctypes.CDLL(str(REPO / "tools/_lab/prefetch_lab.so"))
lab.lab_prefetch.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_void_p, ctypes.c_void_p]

N, K, G = 11008, 4096, 128
dev = torch.device("cuda")
COPIES = 36
qb, sb = N * K // 2, N * (K // G) * 2
per = 2 * (qb + sb)
slabs = []
for c in range(COPIES):
    slab = torch.empty(per, dtype=torch.uint8, device=dev)
    views = []
    off = 0
    for m in range(2):
        q, s = ops.quantize(torch.randn(N, K, device=dev) * 0.02, 0, G)
        qv = slab[off:off + qb].view(N, K // 2)
        qv.copy_(q)
        off += qb
        sv = slab[off:off + sb].view(torch.bfloat16).view(N, K // G)
        sv.copy_(s)
        off += sb
        views += [qv, sv]
    slabs.append((slab, views))
x = torch.randn(K, device=dev).bfloat16()
nw = torch.ones(K, device=dev).bfloat16()
y = torch.empty(N, device=dev, dtype=torch.bfloat16)
sink = torch.zeros(4, dtype=torch.int32, device=dev)


def gemv(i):
    v = slabs[i % COPIES][1]
    ops.q4_gemv_swiglu(x, v[0], v[1], v[2], v[3], N, K, G, 0, norm_weight=nw, out=y)


def pref(i, stream, blocks, unr, pol):
    lab.lab_prefetch(slabs[i % COPIES][0].data_ptr(), per, blocks, unr, pol, sink.data_ptr(), stream)


def timed(build, reps):
    build(reps)  # warm
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        build(reps)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / reps)
    return best


reps = 2 * COPIES


def cold(r):
    for i in range(r):
        gemv(i)


print(f"bytes/launch {per/1e6:.2f} MB", flush=True)
t = timed(cold, reps)
print(f"cold gemv chain          {t:7.2f} us/launch  {per/t/1e3:7.0f} GB/s", flush=True)

for blocks in (64, 256, 1024):
    for unr, pol in ((8, 0), (16, 0), (8, 1)):
        def pre_only(r):
            cur = torch.cuda.current_stream().cuda_stream
            for i in range(r):
                pref(i, cur, blocks, unr, pol)

        def serial(r):
            cur = torch.cuda.current_stream().cuda_stream
            for i in range(r):
                pref(i, cur, blocks, unr, pol)
                gemv(i)

        tp = timed(pre_only, reps)
        ts = timed(serial, reps)
        print(f"blocks={blocks:5d} unr={unr:2d} pol={pol}: prefetch alone {tp:7.2f} us ({per/tp/1e3:6.0f} GB/s); "
              f"prefetch+gemv {ts:7.2f} -> warm gemv {ts - tp:7.2f} us", flush=True)

for blocks in (16, 32, 64, 128):
    for ahead in (1, 2):
        def conc(r, blocks=blocks, ahead=ahead):
            cur = torch.cuda.current_stream()
            side = torch.cuda.Stream()
            side.wait_stream(cur)
            evs = []
            for i in range(ahead):
                pref(i, side.cuda_stream, blocks, 8, 0)
            for i in range(r):
                e0 = torch.cuda.Event()
                e0.record(cur)
                side.wait_event(e0)  # prefetch of i+ahead starts when gemv i starts
                pref(i + ahead, side.cuda_stream, blocks, 8, 0)
                gemv(i)
            cur.wait_stream(side)

        t = timed(conc, reps)
        print(f"concurrent blocks={blocks:4d} ahead={ahead}: {t:7.2f} us/launch  {per/t/1e3:7.0f} GB/s", flush=True)
