#!/bin/bash
# k_postpre: HBM bytes (2 x FETCH_SIZE + WRITE_SIZE per launch, gfx950 correction) and
# duration vs the workgroup count (band height): do the band halo rows cost HBM traffic?
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 1536 3072 6144; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/pph_${b}_$c; rm -rf $d
    PGMG_PP_BLOCKS=$b timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d $d -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline off > $d.log 2>&1 || exit 1
  done
  d=gpurun_out/pph_${b}_trace; rm -rf $d
  PGMG_PP_BLOCKS=$b timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off > $d.log 2>&1 || exit 1
  python3 - "$b" <<'PY'
import csv, glob, sys
b = sys.argv[1]
def per_launch(c):
    f = glob.glob(f"gpurun_out/pph_{b}_{c}/**/*counter_collection.csv", recursive=True)[0]
    v = {}
    for r in csv.DictReader(open(f)):
        if "k_postpre" in r["Kernel_Name"]:
            v.setdefault(r["Dispatch_Id"], 0.0)
            v[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return sum(v.values()) / max(1, len(v)) * 1024
fe, wr = per_launch("FETCH_SIZE"), per_launch("WRITE_SIZE")
f = glob.glob(f"gpurun_out/pph_{b}_trace/**/*kernel_trace.csv", recursive=True)[0]
t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if "k_postpre" in r["Kernel_Name"]]
print(f"blocks {b}: fetch x2 {2 * fe / 1e9:.3f} GB  write {wr / 1e9:.3f} GB  total {(2 * fe + wr) / 1e9:.3f} GB  mean {sum(t) / len(t):.1f} us", flush=True)
PY
done
