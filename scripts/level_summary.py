"""Mean duration per (kernel, grid size) from a rocprofv3 kernel-trace directory."""
import collections
import csv
import glob
import sys

d, label = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    name = r["Kernel_Name"]
    if "pgmg" not in name:
        continue
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    acc[(name.split("(")[0].replace("void pgmg::", ""), g)].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
# levels sharing a grid size (e.g. 8193 and 4097 both at ~2048 workgroups): split by duration
split = {}
for (k, g), v in acc.items():
    s = sorted(v)
    if len(s) >= 4 and s[-1] > 2.5 * s[0]:
        gap = max(range(1, len(s)), key=lambda i: s[i] / s[i - 1])
        split[(k, g, "a")] = s[gap:]
        split[(k, g, "b")] = s[:gap]
    else:
        split[(k, g, "")] = v
acc = split
tot = 0.0
for (k, g, h), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v)
    if sum(v) > 50:
        print(f"  {label:28s} {k[:52]:52s} grid={g:9d}{h:1s} n={len(v):3d} mean={sum(v) / len(v):9.1f}us")
print(f"  {label:28s} TOTAL pgmg kernel time {tot / 1e3:.3f} ms")
