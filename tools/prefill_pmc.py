"""Two 2048-token prefills (cold, then warm) of random-init Llama-2-7B int4-g128 — the bench's prefill — as a short
program for a PMC pass, e.g.

    timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
        -d gpurun_out/pmc_prefill -o pmc -- python tools/prefill_pmc.py

then `python tools/prefill_pmc.py --summarize gpurun_out/pmc_prefill` prints per-kernel MFMA busy fractions of the
warm prefill: SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs) — the share of SIMD cycles
with a matrix instruction in flight while the kernel ran.
"""

from __future__ import annotations

import csv
import sys
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
for p in (str(REPO / "lit-gpt_amd"), str(REPO)):
    if p not in sys.path:
        sys.path.insert(0, p)


def run() -> None:
    import torch

    from generate.base import build_model
    from lit_gpt import Config

    T = 2048
    dev = torch.device("cuda", 0)
    cfg = Config.from_name("Llama-2-7b-hf")
    model = build_model(cfg, quantize="int4-g128", device=dev, max_seq_length=T + 16)
    prompt = torch.randint(0, cfg.vocab_size, (1, T), dtype=torch.int32, device=dev)
    with torch.inference_mode():
        for _ in range(2):
            model(prompt, torch.arange(T, device=dev), last_token_only=True)
            torch.cuda.synchronize()


def summarize(d: Path) -> None:
    """Per kernel name over all its dispatches (the load-time GEMM tuning runs the same shapes as the prefills):
    MFMA busy = sum SQ_VALU_MFMA_BUSY_CYCLES / (sum GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs), and the
    GRBM_GUI_ACTIVE-weighted total over every kernel that issues matrix instructions."""
    rows = [r for f in d.rglob("*counter_collection.csv") for r in csv.DictReader(open(f))]
    by = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(int)
    for r in rows:
        by[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            calls[r["Kernel_Name"]] += 1
    simds = 256 * 4
    tb = tg = 0.0
    print(f"{'kernel':72s} {'calls':>5s} {'GUI_ACTIVE/8':>13s} {'mfma_busy':>10s}")
    for name, c in sorted(by.items(), key=lambda kv: -kv[1].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)):
        b, g = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0), c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if b <= 0 or g <= 0:
            continue
        tb, tg = tb + b, tg + g
        print(f"{name[:72]:72s} {calls[name]:5d} {g:13.0f} {b / (g * simds):10.3f}")
    if tg:
        print(f"{'all MFMA kernels (GUI_ACTIVE-weighted)':72s} {'':5s} {tg:13.0f} {tb / (tg * simds):10.3f}")


def dump(d: Path) -> None:
    """Every counter of a pass, per kernel name, averaged per dispatch (the second, stall-breakdown pass)."""
    rows = [r for f in d.rglob("*counter_collection.csv") for r in csv.DictReader(open(f))]
    by = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(lambda: defaultdict(int))
    for r in rows:
        by[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[r["Kernel_Name"]][r["Counter_Name"]] += 1
    for name, c in sorted(by.items(), key=lambda kv: -max(kv[1].values())):
        print(name[:100])
        for k, v in sorted(c.items()):
            print(f"    {k:28s} {v / max(calls[name][k], 1):16.0f} per dispatch")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(Path(sys.argv[2]))
    elif len(sys.argv) > 2 and sys.argv[1] == "--dump":
        dump(Path(sys.argv[2]))
    else:
        run()
