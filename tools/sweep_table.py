"""Tabulate tools/attn_sweep.py output: rows = splits, columns = positions, one block per library run."""
import re
import sys

tab = []
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sweep.log"):
    if line.startswith("==="):
        tab.append((line.split()[-1].split("/")[-1], {}))
        continue
    m = re.match(r"p=\s*(\d+) splits=\s*(\d+) fused=(\d)\s+([\d.]+) us", line)
    if m and tab:
        tab[-1][1][(int(m[1]), int(m[2]), int(m[3]))] = float(m[4])
for lib, d in tab:
    ps = sorted({k[0] for k in d})
    print(lib, "  p =", ps)
    for sp in sorted({k[1] for k in d}):
        for f in sorted({k[2] for k in d}):
            print(f"  s={sp:3d} f={f} " + "  ".join(f"{d.get((p, sp, f), 0):6.2f}" for p in ps))
