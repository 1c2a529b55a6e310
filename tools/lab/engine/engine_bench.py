"""A/B of the decode step: per-op HIP graph (160 launches) vs the persistent engine (1 launch), Llama-2-7B int4-g128
after a 2048-token prefill, same process and weights (interleaved rounds, MI355X_MICROARCH.md rule 24)."""
import sys, time
from pathlib import Path
REPO = Path(__file__).resolve().parents[3]
sys.path[:0] = [str(Path(__file__).resolve().parent), str(REPO / "lit-gpt_amd"), str(REPO)]
import torch
from generate.base import build_model
from lit_gpt import Config, ops
from lit_gpt.runtime import DecodeGraph
import importlib, os
DecodeEngine = importlib.import_module(os.environ.get("LGA_ENGINE_MOD", "engine2")).DecodeEngine

dev = torch.device("cuda", 0)
T, STEPS = 2048, 64
cfg = Config.from_name("Llama-2-7b-hf", n_layer=int(sys.argv[1]) if len(sys.argv) > 1 else 32)
model = build_model(cfg, quantize="int4-g128", device=dev, max_seq_length=T + 8 * STEPS + 16)
prompt = torch.randint(0, cfg.vocab_size, (T,), generator=torch.Generator().manual_seed(1), dtype=torch.int32).to(dev)
with torch.inference_mode():
    lg = model(prompt.view(1, -1), torch.arange(T, device=dev), last_token_only=True)
    first = ops.argmax(lg.reshape(-1)).to(torch.int32)
    pos = T
    dg = DecodeGraph(model, first, pos, chunk=8)
    pos += 1
    eng = DecodeEngine(model)
    eng.set_embedding(model.transformer.wte.weight[int(first)])
    epos = torch.tensor([pos], device=dev)
    etok = torch.zeros(1, dtype=torch.int32, device=dev)
    eng.step(epos, token=etok)
    ge = torch.cuda.CUDAGraph()
    with torch.cuda.graph(ge):
        for _ in range(8):
            eng.step(epos, token=etok)
    for rnd in range(3):
        for name in ("per-op", "engine"):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(STEPS // 8):
                dg.steps() if name == "per-op" else ge.replay()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / STEPS
            if name == "engine":
                eng.check()
            print(f"round {rnd} {name:7s} {dt * 1e6:8.1f} us/step  {1 / dt:7.1f} tok/s", flush=True)
