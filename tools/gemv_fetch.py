"""HBM bytes per launch (PMC FETCH_SIZE) of the decode step's weaker GEMVs at Llama-2-7B int4-g128 shape — qkv
(RMSNorm fused), attn.proj (+ residual), mlp.proj (K = 11008, + residual) — against their algorithmic bytes.

usage: python tools/gemv_fetch.py          (runs itself under `rocprofv3 --pmc FETCH_SIZE` as a child process,
                                             before this process touches the GPU; MI355X_MICROARCH.md HBM section:
                                             FETCH_SIZE KiB x 2 on gfx950)
Each GEMV runs once on each of 24 distinct weight sets (well past the 256 MB Infinity Cache), so every launch
streams its weights from HBM as in the decode step.
"""

import csv
import shutil
import statistics
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
SHAPES = {  # name: (N, K, norm, residual)
    "qkv": (12288, 4096, True, False),
    "attn.proj": (4096, 4096, False, True),
    "mlp.proj": (4096, 11008, False, True),
}


def algorithmic_bytes(N, K, norm, res, group=128):
    return N * K // 2 + N * (K // group) * 2 + K * 2 + (K * 2 if norm else 0) + (N * 2 if res else 0) + N * 2


def child():
    import torch

    sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
    from lit_gpt import ops

    dev = torch.device("cuda")
    for name, (N, K, norm, res) in SHAPES.items():
        sets = [ops.quantize(torch.randn(N, K, device=dev) * 0.02, 0, 128) for _ in range(24)]
        x = torch.randn(K, device=dev).bfloat16()
        nw = torch.ones(K, device=dev).bfloat16() if norm else None
        r = torch.randn(N, device=dev).bfloat16() if res else None
        out = torch.empty(N, dtype=torch.bfloat16, device=dev)
        torch.cuda.synchronize()
        for qw, sc in sets:
            ops.q4_gemv(x, qw, sc, N, K, 128, 0, norm_weight=nw, residual=r, out=out)
        torch.cuda.synchronize()
        del sets


def main():
    if "--child" in sys.argv:
        return child()
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    out = Path(tempfile.mkdtemp(prefix="lga_fetch_"))
    cmd = [exe, "--pmc", "FETCH_SIZE", "--output-format", "csv", "-d", str(out), "-o", "pmc", "--",
           sys.executable, str(Path(__file__).resolve()), "--child"]
    subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=300, check=True)
    rows = [r for f in out.rglob("*counter_collection.csv") for r in csv.DictReader(open(f))
            if r.get("Counter_Name") == "FETCH_SIZE"]
    by = {}
    for r in rows:
        by.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    # launch order: 24 qkv, then 24 attn.proj, then 24 mlp.proj; the kernels differ by template arguments
    order = {"gemv_q4_kernel<4, 2, 0, false, true, false>": "qkv",
             "gemv_q4_kernel<4, 2, 0, false, false, true>": "attn.proj",
             "gemv_q4_kernel<2, 6, 0, false, false, true>": "mlp.proj"}
    for kname, vals in by.items():
        name = next((v for k, v in order.items() if k in kname), None)
        if name is None:
            continue
        N, K, norm, res = SHAPES[name]
        alg = algorithmic_bytes(N, K, norm, res)
        kib = statistics.median(vals)
        print(f"{name:10s} {kname[:60]:60s} launches {len(vals):3d}  FETCH_SIZE x2 = {2 * kib * 1024 / 1e6:7.2f} MB"
              f"  algorithmic {alg / 1e6:7.2f} MB  ratio {2 * kib * 1024 / alg:.3f}", flush=True)
    shutil.rmtree(out, ignore_errors=True)


if __name__ == "__main__":
    main()
