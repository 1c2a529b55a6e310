"""Lab probe: overlap the decode attention's K/V stream with the qkv GEMV that precedes it (two graph branches).

Llama-2-7B geometry, 32 "layers" with distinct buffers (no cache reuse across layers):
  qkv GEMV      12288 x 4096 int4-g128 (+ fused RMSNorm)          26 MB per layer
  K/V stream    2 x 32 groups x 2200 keys x 128 x bf16               36 MB per layer
Prints us per layer for: GEMV alone, K/V read alone, both sequential, both on concurrent branches, and the
"prefetch K/V into registers, wait for the GEMV's flag" shape.

usage: python tools/overlap_lab.py     (needs tools/_lab/overlap_lab.so, see tools/overlap_lab.hip)
"""
import ctypes
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
from lit_gpt import ops  # noqa: E402

lab = ctypes.CDLL(str(REPO / "tools/_lab/overlap_lab.so"))
V, L, I = ctypes.c_void_p, ctypes.c_long, ctypes.c_int
lab.lab_set.argtypes = [V, ctypes.c_uint, V]
lab.lab_spin.argtypes = [V, V, V]
lab.lab_read.argtypes = [V, L, I, I, V, V]
lab.lab_prefetch_wait.argtypes = [V, L, I, V, V, V, V, V]

dev = torch.device("cuda")
LAYERS, N, K, G = 32, 12288, 4096, 128
KV = 2 * 32 * 2200 * 128 * 2
W = [ops.quantize(torch.randn(N, K, device=dev) * 0.02, 0, G) for _ in range(LAYERS)]
kv = [torch.empty(KV, dtype=torch.uint8, device=dev).random_(0, 255) for _ in range(LAYERS)]
x = torch.randn(K, device=dev).bfloat16()
nw = torch.ones(K, device=dev).bfloat16()
y = torch.empty(N, device=dev, dtype=torch.bfloat16)
sink = torch.zeros(4, dtype=torch.int32, device=dev)
flags = torch.zeros(LAYERS, 64, dtype=torch.int32, device=dev)  # one 256-B line per layer
done = torch.zeros(LAYERS, 64, dtype=torch.int32, device=dev)
err = torch.zeros(1, dtype=torch.int32, device=dev)


def cur():
    return torch.cuda.current_stream().cuda_stream


def gemv(l):
    ops.q4_gemv(x, W[l][0], W[l][1], N, K, G, 0, norm_weight=nw, out=y)


def read(l, stream, blocks=256, unr=8):
    lab.lab_read(kv[l].data_ptr(), KV, blocks, unr, sink.data_ptr(), stream)


def timed(build, reps=3):
    build()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        build()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(reps):
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / LAYERS)
    return best


def fork_join(body):
    def run():
        main = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(main)
        body(main, side)
        main.wait_stream(side)
    return run


# 1. are two graph branches concurrent?  side: spin until main sets the flag
def conc(main, side):
    for l in range(LAYERS):
        e0 = torch.cuda.Event()
        e0.record(main)
        side.wait_event(e0)
        lab.lab_spin(flags[l].data_ptr(), err.data_ptr(), side.cuda_stream)
        gemv(l)
        lab.lab_set(flags[l].data_ptr(), 1, main.cuda_stream)


err.zero_()
t = timed(fork_join(conc))
torch.cuda.synchronize()
print(f"concurrency probe: {t:7.2f} us/layer, spin timeouts {int(err.item())} (0 = branches run concurrently)",
      flush=True)
flags.zero_()

tg = timed(lambda: [gemv(l) for l in range(LAYERS)])
print(f"qkv GEMV alone                 {tg:7.2f} us  ({26e6 / tg / 1e3:6.0f} GB/s)", flush=True)
for blocks, unr in ((256, 8), (512, 8), (1024, 8), (256, 16), (512, 4)):
    tr = timed(lambda: [read(l, cur(), blocks, unr) for l in range(LAYERS)])
    print(f"K/V read alone blocks={blocks:4d} unr={unr:2d}  {tr:7.2f} us  ({KV / tr / 1e3:6.0f} GB/s)", flush=True)
ts = timed(lambda: [(gemv(l), read(l, cur())) for l in range(LAYERS)])
print(f"GEMV then read (sequential)    {ts:7.2f} us", flush=True)


def overlap(main, side):
    for l in range(LAYERS):
        e0 = torch.cuda.Event()
        e0.record(main)
        side.wait_event(e0)
        read(l, side.cuda_stream)
        gemv(l)
        e1 = torch.cuda.Event()
        e1.record(side)
        main.wait_event(e1)


print(f"GEMV || read (branches)        {timed(fork_join(overlap)):7.2f} us", flush=True)

for nl in (16, 32, 64):
    def pw(main, side, nl=nl):
        for l in range(LAYERS):
            e0 = torch.cuda.Event()
            e0.record(main)
            side.wait_event(e0)
            lab.lab_prefetch_wait(kv[l].data_ptr(), KV, nl, flags[l].data_ptr(), done[l].data_ptr(),
                                  err.data_ptr(), sink.data_ptr(), side.cuda_stream)
            gemv(l)
            lab.lab_set(flags[l].data_ptr(), 1, main.cuda_stream)
            e1 = torch.cuda.Event()
            e1.record(side)
            main.wait_event(e1)

    err.zero_()
    t = timed(fork_join(pw))
    torch.cuda.synchronize()
    print(f"GEMV || prefetch-wait nl={nl:2d}   {t:7.2f} us  (timeouts {int(err.item())})", flush=True)

    def pw_alone(nl=nl):
        for l in range(LAYERS):
            lab.lab_set(flags[l].data_ptr(), 1, cur())
            lab.lab_prefetch_wait(kv[l].data_ptr(), KV, nl, flags[l].data_ptr(), done[l].data_ptr(),
                                  err.data_ptr(), sink.data_ptr(), cur())

    print(f"prefetch-wait alone nl={nl:2d}     {timed(pw_alone):7.2f} us", flush=True)
