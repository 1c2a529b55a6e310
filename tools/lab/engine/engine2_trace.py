"""Per-op timeline of the persistent decode engine version 2 (lab build with -DLGA_ENGINE_TRACE:
make -C lit-gpt_amd/csrc lab-engine2 LABFLAGS=-DLGA_ENGINE_TRACE LAB2=../../tools/_lab/liblga_engine2_trace.so).
Runs a few engine steps of Llama-2-7B int4-g128 after a 2048-token prefill and prints, per op of one step, the
median / max over CUs (us after the launch's first event) of: the gather waves' start, input edge complete,
staging done; compute wave 0's first tile and op done. Saves the raw events to gpurun_out/engine2_trace.npy."""
import ctypes, os, sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[3]
os.environ["LGA_ENGINE2_LIB"] = sys.argv[2] if len(sys.argv) > 2 else str(REPO / "tools" / "_lab" / "liblga_engine2_trace.so")
sys.path[:0] = [str(Path(__file__).resolve().parent), str(REPO / "lit-gpt_amd"), str(REPO)]
import numpy as np
import torch
from generate.base import build_model
from lit_gpt import Config
from engine2 import DecodeEngine, engine_library

dev = torch.device("cuda", 0)
L = int(sys.argv[1]) if len(sys.argv) > 1 else 32
T = 2048
cfg = Config.from_name("Llama-2-7b-hf", n_layer=L)
model = build_model(cfg, quantize="int4-g128", device=dev, max_seq_length=T + 64)
lib = engine_library()
lib.lga_engine_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_long]
TR_OPS, TR_EV, NCU = 192, 8, 256
buf = np.zeros(NCU * TR_OPS * TR_EV, dtype=np.uint64)
names = ["qkv", "attn", "oproj", "fc", "down"]
import time
with torch.inference_mode():
    prompt = torch.randint(0, cfg.vocab_size, (T,), dtype=torch.int32).to(dev)
    lg = model(prompt.view(1, -1), torch.arange(T, device=dev), last_token_only=True)
    eng = DecodeEngine(model)
    eng.set_embedding(model.transformer.wte.weight[int(torch.argmax(lg.reshape(-1).float()))])
    pos = torch.tensor([T], device=dev)
    for it in range(4):
        lib.lga_engine_trace_read(buf.ctypes.data, buf.size)  # clear
        torch.cuda.synchronize()
        t = time.perf_counter()
        eng.step(pos)
        torch.cuda.synchronize()
        print(f"launch {it}: {(time.perf_counter() - t) * 1e6:.1f} us wall", flush=True)
        lib.lga_engine_trace_read(buf.ctypes.data, buf.size)
    eng.check()
tr = buf.reshape(NCU, TR_OPS, TR_EV).astype(np.int64)
out = Path(os.environ.get("GRAFT_REPO_ROOT", REPO)) / "gpurun_out" / "engine2_trace.npy"
out.parent.mkdir(exist_ok=True)
np.save(out, tr)
nops = L * 5 + 1
valid = tr[tr > 0]
t0 = valid.min()
def col(k, e):
    v = tr[:, k, e]
    v = v[v > 0]
    return (v - t0) / 100.0 if v.size else np.array([np.nan])
last = max(np.nanmax(col(k, 7)) for k in range(nops))
print(f"step (first event -> last op done on compute wave 0): {last:.1f} us")
print("op         gw start  edge ok (med/max)   staged (med/max) | cw0 first tile (med/max)  cw0 done (med/max) | attn: parts published combined")
for k in list(range(min(nops, 15))) + list(range(max(15, nops - 6), nops)):
    name = names[k % 5] if k < L * 5 else "lm"
    f = lambda e: (np.nanmedian(col(k, e)), np.nanmax(col(k, e)))
    s = f"{k:3d} {name:6s} {f(0)[0]:8.1f}  {f(1)[0]:8.1f}/{f(1)[1]:7.1f}  {f(5)[0]:8.1f}/{f(5)[1]:7.1f} | {f(6)[0]:8.1f}/{f(6)[1]:7.1f}  {f(7)[0]:8.1f}/{f(7)[1]:7.1f}"
    if name == "attn":
        s += f" | {f(2)[0]:7.1f} {f(3)[0]:7.1f} {f(4)[1]:7.1f}"
    print(s)
per_layer = [(np.nanmedian(col(5 * l + 5, 7)) - np.nanmedian(col(5 * l, 7))) for l in range(L - 1)]
print("per-layer (median op-done delta over 5 ops):", " ".join(f"{v:.1f}" for v in per_layer[:8]), "... mean", f"{np.mean(per_layer):.1f} us")
