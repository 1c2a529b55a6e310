"""Per-call time of the fused row-parallel GEMV + all-reduce (lga_q4_gemv_allreduce) vs lga_q4_gemv +
lga_allreduce_bf16, for the 7B attn.proj / mlp.proj shards at TP = 2, 4, 8 — all ranks as processes on ONE GPU
(the only setup this box has), so the numbers compare the two forms on a shared device, not multi-GPU latency.
usage: python tools/tp_fused_time.py  (writes gpurun_out/tp_fused_time.txt)"""
import os
import socket
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
out_all = REPO / "gpurun_out" / "tp_fused_time.txt"
out_all.parent.mkdir(exist_ok=True)
lines = []
for n in (2, 4, 8):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    tmp = REPO / "gpurun_out" / f"tp_fused_time_{n}.txt"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(REPO / "tests" / "workers" / "gemv_allreduce_worker.py"),
           str(tmp), "--time"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=dict(os.environ, OMP_NUM_THREADS="2"))
    if r.returncode:
        print(r.stderr[-3000:])
        sys.exit(r.returncode)
    lines.append(tmp.read_text())
    print(lines[-1], end="", flush=True)
out_all.write_text("".join(lines))
