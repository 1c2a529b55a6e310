"""SQ / TCC counters of the decode attention at two geometries (one rocprofv3 --pmc pass each, run as a child
process): Mixtral at p = 32066 (32 splits, q_per_kv 4) and Llama-2-7B at p = 2302 (8 splits, q_per_kv 1).

usage: python tools/attn_pmc.py [--mem]    (the parent never touches the GPU; each pass is `timeout -s KILL`-bounded)
Counters (gfx950 slots: SQ <= 8, TCC <= 4): SQ_WAVE_CYCLES, SQ_WAIT_ANY (parked on s_waitcnt / barrier),
SQ_WAIT_INST_ANY (issue stall), SQ_ACTIVE_INST_ANY, SQ_ACTIVE_INST_VALU, SQ_INSTS_VALU, TCC_HIT_sum, TCC_MISS_sum.
"""

import csv
import math
import shutil
import statistics
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
GEOMS = {"mixtral_p32066": (32, 8, 32768, 32066, 24), "llama7b_p2302": (32, 32, 2304, 2302, 32)}
COUNTERS = ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
            "SQ_INSTS_VALU", "TCC_HIT_sum", "TCC_MISS_sum"]
# --mem: the vector-memory path instead (TA <= 2, TCP <= 4, GRBM <= 2 per pass): texture-address busy and its stall on
# the L1 (TC), the per-CU L1 -> L2 read request count and summed latency (cycles), L1 pending stalls, kernel cycles
MEM_COUNTERS = ["TA_TA_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TCP_TCC_READ_REQ_sum",
                "TCP_TCC_READ_REQ_LATENCY_sum", "TCP_PENDING_STALL_CYCLES_sum", "GRBM_GUI_ACTIVE"]
if "--mem" in sys.argv:
    COUNTERS = MEM_COUNTERS


def child(name):
    import torch

    sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
    from lit_gpt import ops

    H, G, S, p, layers = GEOMS[name]
    hs, dev = 128, torch.device("cuda")
    caches = [(torch.randn(G, S, hs, device=dev).bfloat16(), torch.randn(G, S, hs, device=dev).bfloat16())
              for _ in range(layers)]
    qkv = torch.randn(1, (H + 2 * G) * hs, device=dev).bfloat16()
    cos, sin = torch.randn(S, hs, device=dev), torch.randn(S, hs, device=dev)
    splits = ops.decode_splits(G, H // G, hs, S)
    ws = ops.AttentionWorkspace(1, H, G, hs, splits, dev)
    pos = torch.tensor([p], device=dev)
    torch.cuda.synchronize()
    for kc, vc in caches:
        ops.attention_decode_fused(qkv, kc, vc, pos, pos, cos, sin, H, G, hs, hs, 1.0 / math.sqrt(hs), splits,
                                   workspace=ws)
    torch.cuda.synchronize()


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        return child(sys.argv[2])
    extra = ["--mem"] if "--mem" in sys.argv else []
    if "--gemv" in sys.argv:  # the decode GEMVs instead (tools/gemv_fetch.py's launches), per kernel
        return gemv_pass()
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    for name in GEOMS:
        out = Path(tempfile.mkdtemp(prefix="lga_apmc_"))
        cmd = ["timeout", "-s", "KILL", "90", exe, "--pmc", *COUNTERS, "--output-format", "csv", "-d", str(out),
               "-o", "pmc", "--", sys.executable, str(Path(__file__).resolve()), "--child", name, *extra]
        r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
        if r.returncode != 0:
            print(f"{name}: rocprofv3 pass failed ({r.returncode}): {r.stderr[-400:]}", flush=True)
            return 1
        rows = [row for f in out.rglob("*counter_collection.csv") for row in csv.DictReader(open(f))
                if "attn_kernel" in row.get("Kernel_Name", "")]
        med = {c: statistics.median(float(rw["Counter_Value"]) for rw in rows if rw["Counter_Name"] == c)
               for c in COUNTERS if any(rw["Counter_Name"] == c for rw in rows)}
        wc = med.get("SQ_WAVE_CYCLES", float("nan"))
        print(f"{name}: " + "  ".join(f"{c} {v:.4g}" for c, v in med.items()), flush=True)
        if COUNTERS is MEM_COUNTERS:
            gui = med["GRBM_GUI_ACTIVE"]
            print(f"   per CU-cycle (256 CUs x GRBM_GUI_ACTIVE): TA busy {med['TA_TA_BUSY_sum'] / (256 * gui):.3f}  "
                  f"TA addr stalled by L1 {med['TA_ADDR_STALLED_BY_TC_CYCLES_sum'] / (256 * gui):.3f}  "
                  f"L1 pending stall {med['TCP_PENDING_STALL_CYCLES_sum'] / (256 * gui):.3f};  L1->L2 read latency "
                  f"{med['TCP_TCC_READ_REQ_LATENCY_sum'] / max(med['TCP_TCC_READ_REQ_sum'], 1):.0f} cycles over "
                  f"{med['TCP_TCC_READ_REQ_sum']:.4g} requests", flush=True)
            shutil.rmtree(out, ignore_errors=True)
            continue
        print(f"   per wave-cycle: wait_any {med['SQ_WAIT_ANY'] / wc:.3f}  wait_inst {med['SQ_WAIT_INST_ANY'] / wc:.3f}"
              f"  active_any {med['SQ_ACTIVE_INST_ANY'] / wc:.3f}  active_valu {med['SQ_ACTIVE_INST_VALU'] / wc:.3f};"
              f"  L2 hit {med['TCC_HIT_sum'] / (med['TCC_HIT_sum'] + med['TCC_MISS_sum']):.3f}", flush=True)
        shutil.rmtree(out, ignore_errors=True)


def gemv_pass():
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    out = Path(tempfile.mkdtemp(prefix="lga_gpmc_"))
    cmd = ["timeout", "-s", "KILL", "120", exe, "--pmc", *COUNTERS, "--output-format", "csv", "-d", str(out),
           "-o", "pmc", "--", sys.executable, str(REPO / "tools" / "gemv_fetch.py"), "--child"]
    r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    if r.returncode != 0:
        print(f"gemv: rocprofv3 pass failed ({r.returncode}): {r.stderr[-400:]}", flush=True)
        return 1
    rows = [row for f in out.rglob("*counter_collection.csv") for row in csv.DictReader(open(f))
            if "gemv" in row.get("Kernel_Name", "")]
    for kname in sorted({rw["Kernel_Name"] for rw in rows}):
        med = {c: statistics.median(float(rw["Counter_Value"]) for rw in rows
                                    if rw["Counter_Name"] == c and rw["Kernel_Name"] == kname) for c in COUNTERS}
        wc = med["SQ_WAVE_CYCLES"]
        print(f"{kname[:64]}: wait_any {med['SQ_WAIT_ANY'] / wc:.3f}  wait_inst {med['SQ_WAIT_INST_ANY'] / wc:.3f}"
              f"  active_any {med['SQ_ACTIVE_INST_ANY'] / wc:.3f}  active_valu {med['SQ_ACTIVE_INST_VALU'] / wc:.3f}"
              f"  insts_valu {med['SQ_INSTS_VALU']:.4g}  L2 hit "
              f"{med['TCC_HIT_sum'] / (med['TCC_HIT_sum'] + med['TCC_MISS_sum']):.3f}", flush=True)
    shutil.rmtree(out, ignore_errors=True)


if __name__ == "__main__":
    sys.exit(main())
