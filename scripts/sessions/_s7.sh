set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_cross.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_fcycle.py tests/test_gpu_strips.py tests/test_gpu_recompute.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t7.log 2>&1; rc=$?; tail -3 gpurun_out/t7.log; [ $rc -eq 0 ] || exit $rc
for v in base new base new; do
  if [ $v = base ]; then LIB=$L/libpgmg_base.so; else LIB=$L/libpgmg.so; fi
  PGMG_LIB=$LIB timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/st_$v -o run -- python3 scripts/vrun.py 16385 20 > gpurun_out/st_$v.log 2>&1 || exit 1
  python3 - $v <<'P'
import csv, glob, sys
v = sys.argv[1]
f = glob.glob(f'gpurun_out/st_{v}/**/run_kernel_trace.csv', recursive=True)[0]
import collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r['Kernel_Name'].replace('void pgmg::', '')[:48]
    acc[(n, r['Grid_Size_X'], r['Grid_Size_Y'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
tot = 0
for k, x in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    if len(x) >= 20 and 'rocclr' not in k[0]:
        print(f"{v:5s} {sum(x)/len(x):9.2f} us n={len(x):3d} {k[0]} {k[1]}x{k[2]}")
P
done
