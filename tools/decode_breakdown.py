"""Per-decode-step kernel breakdown from a rocprofv3 --kernel-trace CSV (argmax kernels delimit steps)."""
import collections
import csv
import sys

path = sys.argv[1]
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 32
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "argmax" in r["Kernel_Name"]]
a, b = idx[-nsteps - 1], idx[-1]
seg = rows[a + 1:b + 1]
d = collections.defaultdict(list)
for r in seg:
    d[r["Kernel_Name"].split("(")[0][:70]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = 0
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:70s} n/step={len(v)/nsteps:5.1f} avg={sum(v)/len(v)/1e3:8.2f}us per_step={sum(v)/nsteps/1e3:8.1f}us")
    tot += sum(v)
span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / nsteps / 1e3
print(f"kernel sum per step {tot/nsteps/1e3:.1f} us; wall per step {span:.1f} us")
