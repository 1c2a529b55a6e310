"""Per-op timeline of the persistent decode engine (lab build with -DLGA_ENGINE_TRACE: make -C lit-gpt_amd/csrc
lab-engine LABFLAGS=-DLGA_ENGINE_TRACE LAB=../../tools/_lab/liblga_engine_trace.so). Runs a few engine steps of Llama-2-7B int4-g128 after a 2048-token prefill and prints, per op of one
step, the spread over CUs of: counter wait, gather, unit compute, publish, and the loader's issue window."""
import ctypes, os, sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[3]
os.environ["LGA_ENGINE_LIB"] = sys.argv[3] if len(sys.argv) > 3 else str(REPO / "tools" / "_lab" / "liblga_engine_trace.so")
sys.path[:0] = [str(Path(__file__).resolve().parent), str(REPO / "lit-gpt_amd"), str(REPO)]
import numpy as np
import torch
from generate.base import build_model
from lit_gpt import Config, ops
from engine import DecodeEngine, engine_library

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
with torch.inference_mode():
    prompt = torch.randint(0, cfg.vocab_size, (T,), dtype=torch.int32).to(dev)
    lg = model(prompt.view(1, -1), torch.arange(T, device=dev), last_token_only=True)
    eng = DecodeEngine(model)
    eng.set_embedding(model.transformer.wte.weight[int(torch.argmax(lg.reshape(-1).float()))])
    pos = torch.tensor([T], device=dev)
    mode = sys.argv[2] if len(sys.argv) > 2 else "full"
    import time
    for it in range(4):
        lib.lga_engine_trace_read(buf.ctypes.data, buf.size)  # clear
        torch.cuda.synchronize()
        t = time.perf_counter()
        eng.step(pos, op_limit={"stream": -1, "stream_il": -2}.get(mode, 0))
        torch.cuda.synchronize()
        print(f"launch {it}: {(time.perf_counter() - t) * 1e6:.1f} us wall", flush=True)
        lib.lga_engine_trace_read(buf.ctypes.data, buf.size)
        if mode.startswith("stream"):
            pos.fill_(T)
    eng.check()
tr = buf.reshape(NCU, TR_OPS, TR_EV).astype(np.int64)
out = Path(os.environ.get("GRAFT_REPO_ROOT", REPO)) / "gpurun_out" / "engine_trace.npy"
out.parent.mkdir(exist_ok=True)
np.save(out, tr)
nops = L * 5 + 1
t0 = tr[:, 0, 0][tr[:, 0, 0] > 0].min()
rel = lambda v: (v - t0) / 100.0  # us
print(f"step wall (first gather -> last publish / drain): {rel(max(tr[:, nops - 1, 4].max(), tr[:, nops - 1, 3].max())):.1f} us")
print("op        gatherStart  ctrOK   gathered  unitsDone  published  | wait  gather units   | loader: first..last line")
for k in list(range(min(nops, 12))) + [nops - 6, nops - 5, nops - 4, nops - 3, nops - 2, nops - 1]:
    e = tr[:, k, :]
    name = names[k % 5] if k < L * 5 else "lm"
    med = lambda i: np.median(rel(e[:, i]))
    mx = lambda i: rel(e[:, i]).max()
    print(f"{k:3d} {name:6s} {med(0):9.1f} {med(1):8.1f} {med(2):9.1f} {med(3):10.1f} {mx(4):10.1f} | "
          f"{np.median(e[:,1]-e[:,0])/100:5.2f} {np.median(e[:,2]-e[:,1])/100:5.2f} {np.median(e[:,3]-e[:,2])/100:6.2f} | "
          f"{med(5):8.1f} .. {med(6):8.1f}")

# per-CU skew: which CUs finish each op's units last, and is it the same CUs every op
print("\nper-op spread of unitsDone over CUs (us after the median) and the 8 latest CUs")
late_count = np.zeros(NCU, dtype=int)
for k in range(nops):
    d = rel(tr[:, k, 3])
    d = d - np.median(d)
    order = np.argsort(d)[::-1]
    late_count[order[:16]] += 1
    if k < 15 or k >= nops - 6:
        print(f"{k:3d} {(names[k % 5] if k < L * 5 else 'lm'):6s} p90 {np.percentile(d, 90):6.2f} p99 {np.percentile(d, 99):6.2f} "
              f"max {d.max():6.2f} | late CUs {list(order[:8])}")
top = np.argsort(late_count)[::-1][:24]
print("CUs most often among the 16 latest (count over", nops, "ops):", [(int(c), int(late_count[c])) for c in top])
print("by blockIdx % 8:", [int(late_count[np.arange(NCU) % 8 == x].sum()) for x in range(8)])
print("attention split of the late CUs (c // G):", [int(c) // 32 for c in top])
