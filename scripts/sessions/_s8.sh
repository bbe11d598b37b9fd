set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
for v in base new nopf nopf3 base new nopf nopf3; do
  case $v in base) LIB=$L/libpgmg_base.so;; new) LIB=$L/libpgmg.so;; *) LIB=$L/libpgmg_$v.so;; esac
  PGMG_LIB=$LIB timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s8_$v -o run -- python3 scripts/vrun.py 16385 20 > gpurun_out/s8_$v.log 2>&1 || exit 1
  python3 - $v <<'P'
import csv, glob, sys, collections
v = sys.argv[1]
f = sorted(glob.glob(f'gpurun_out/s8_{v}/**/run_kernel_trace.csv', recursive=True))[-1]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r['Kernel_Name'].replace('void pgmg::', '')[:14]
    acc[(n, r['Grid_Size_X'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
out = []
for k, x in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    if len(x) >= 20 and 'rocclr' not in k[0] and sum(x)/len(x) > 9:
        out.append(f"{k[0][2:8]}{k[1]}:{sum(x)/len(x):.1f}")
print(v, ' '.join(out))
P
done
