"""Lab probe (tools/chain_lab.hip): a chain of 64 streaming kernels (26 MB each, the qkv GEMV's bytes), one
stream with stream-order dependencies vs two alternating streams with device-counter hand-offs.

usage: python tools/chain_lab.py     (needs tools/_lab/chain_lab.so)
"""
import ctypes
import sys
import time
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
lab = ctypes.CDLL(str(REPO / "tools/_lab/chain_lab.so"))
P = ctypes.c_void_p
lab.lab_chain.argtypes = [P, ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_int, P, P, P, P, P, ctypes.c_uint]

dev = torch.device("cuda")
N = 64
for mb in (8, 26, 46):
    nbytes = mb << 20
    bufs = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(N)]
    ptrs = (P * N)(*[b.data_ptr() for b in bufs])
    ctr = torch.zeros(N * 64, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    for blocks in (256, 512, 1024):
        res = {}
        for mode in (0, 1):
            best = 1e9
            for rep in range(6):
                ctr.zero_()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                lab.lab_chain(ptrs, N, nbytes, blocks, mode, ctr.data_ptr(), err.data_ptr(), sink.data_ptr(),
                              s0.cuda_stream, s1.cuda_stream, 0)
                torch.cuda.synchronize()
                if rep:
                    best = min(best, (time.perf_counter() - t0) * 1e6 / N)
            res[mode] = best
        print(f"{mb:3d} MB blocks={blocks:5d}: one stream {res[0]:7.2f} us/kernel ({nbytes / res[0] / 1e3:5.0f} GB/s), "
              f"two streams + counters {res[1]:7.2f} us ({nbytes / res[1] / 1e3:5.0f} GB/s), timeouts "
              f"{int(err.item())}", flush=True)
    del bufs
    torch.cuda.empty_cache()
