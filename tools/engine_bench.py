"""A/B of the decode step: per-op HIP graph (160 launches) vs the persistent engine (1 launch), Llama-2-7B int4-g128
after a 2048-token prefill, same process and weights (interleaved rounds, MI355X_MICROARCH.md rule 24)."""
import sys, time
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
import torch
from generate.base import build_model
from lit_gpt import Config, ops
from lit_gpt.runtime import DecodeGraph

dev = torch.device("cuda", 0)
T, STEPS = 2048, 64
cfg = Config.from_name("Llama-2-7b-hf", n_layer=int(sys.argv[1]) if len(sys.argv) > 1 else 32)
model = build_model(cfg, quantize="int4-g128", device=dev, max_seq_length=T + 8 * STEPS + 16)
prompt = torch.randint(0, cfg.vocab_size, (T,), generator=torch.Generator().manual_seed(1), dtype=torch.int32).to(dev)
with torch.inference_mode():
    lg = model(prompt.view(1, -1), torch.arange(T, device=dev), last_token_only=True)
    first = ops.argmax(lg.reshape(-1)).to(torch.int32)
    pos = T
    graphs = {}
    for name, eng in (("per-op", False), ("engine", True)):
        graphs[name] = DecodeGraph(model, first, pos, chunk=8, engine=eng)
        pos += 1
    for rnd in range(3):
        for name, dg in graphs.items():
            dg.pos.fill_(pos)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(STEPS // 8):
                dg.steps()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / STEPS
            if dg.engine is not None:
                dg.check()
            print(f"round {rnd} {name:7s} {dt * 1e6:8.1f} us/step  {1 / dt:7.1f} tok/s  (pos {pos})", flush=True)
            pos += STEPS
