"""Lab: phase timeline of the device sampler (csrc/sample.hip, lab build with -DLGA_SAMPLE_TRACE).

    make -C lit-gpt_amd/csrc lab-lib LABSRC=sample LABFLAGS=-DLGA_SAMPLE_TRACE LABLIB=../../tools/_fa/libsample_trace.so
    python tools/sample_trace.py tools/_fa/libsample_trace.so

Times one top-k 200 / temperature 0.8 draw over 32000 bf16 logits shaped like a decode step's (N(0, 3)), then prints
thread 0's timestamps (100 MHz clock, so 10 ns resolution) after: staging, max, select, kept set, softmax, draw.
"""
import ctypes
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
from lit_gpt import ops  # noqa: E402


def main(lib_path: str) -> None:
    ops._lib = ops.load_library(Path(lib_path))
    lib = ctypes.CDLL(lib_path)
    dev = torch.device("cuda")
    names = ["staged", "max", "select", "kept set", "softmax", "draw"]
    for label, x in (("N(0,3)", torch.randn(32000, generator=torch.Generator().manual_seed(0)) * 3),
                     ("peaked", torch.randn(32000, generator=torch.Generator().manual_seed(1)))):
        if label == "peaked":
            x[123] = 1000.0
        x = x.bfloat16().to(dev)
        counter = torch.zeros(1, dtype=torch.int64, device=dev)
        for _ in range(20):
            ops.sample_topk(x, 200, 0.8, seed=1, counter=counter)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 16)()
        assert lib.lga_sample_trace(buf) == 0
        t0 = buf[0]
        row = "  ".join(f"{n} {(buf[i] - t0) * 10 / 1000:6.2f}" for i, n in enumerate(names))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(100):
            ops.sample_topk(x, 200, 0.8, seed=1, counter=counter)
        e1.record()
        torch.cuda.synchronize()
        print(f"{label:7s} launch {e0.elapsed_time(e1) * 10:6.2f} us | us after staging: {row}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
