"""Phase timeline of one lga_decode_layer launch (lab build with -DLGA_LAYER_TRACE).

usage: LAYER_LIB=tools/_lab/ltrace.so python tools/layer_trace.py [prompt_len]
Stamps (thread 0 = control wave, us from the earliest workgroup start): 0 start, 1 S1 input staged, 2 S1 done,
3 S2 input ready, 4 S2 done, 5 S3 input ready, 6 S3 done, 7 S4 input ready, 8 S4 done, 9 S5 input ready, 10 end.
"""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
from lit_gpt import ops  # noqa: E402


@torch.inference_mode()
def main(T=2048):
    lib = ops.load_library(Path(os.environ["LAYER_LIB"]))
    ops._lib = lib
    lib.lga_layer_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    from generate.base import build_model
    from lit_gpt import Config

    dev = torch.device("cuda")
    cfg = Config.from_name("Llama-2-7b-hf", n_layer=16, vocab_size=512, padding_multiple=64, block_size=4096)
    model = build_model(cfg, quantize="int4-g128", device=dev, seed=7, max_seq_length=T + 8)
    ids = torch.randint(0, 500, (T + 4,), device=dev)
    model(ids[:T].view(1, -1), torch.arange(T, device=dev), last_token_only=True)
    for i in range(3):
        model(ids[T + i:T + i + 1].view(1, 1), torch.tensor([T + i], device=dev))
    torch.cuda.synchronize()
    NB = ops.num_cus()
    buf = np.zeros(NB * 16, dtype=np.uint64)
    lib.lga_layer_trace_read(buf.ctypes.data, NB * 16)
    tr = buf.reshape(NB, 16).astype(np.int64)
    t0 = tr[:, 0].min()
    rel = (tr - t0) / 100.0
    names = ["start", "S1 x staged", "S1 done", "S2 in ready", "S2 done", "S3 in ready", "S3 done", "S4 in ready",
             "S4 done", "S5 in ready", "end"]
    for k, n in enumerate(names):
        q = np.percentile(rel[:, k], [0, 50, 100])
        print(f"  {n:12s} min {q[0]:7.2f}  med {q[1]:7.2f}  max {q[2]:7.2f}")


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
