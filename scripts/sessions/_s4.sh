set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
for b in 3072 512; do
  PGMG_LIB=$L/libpgmg_ab.so PGMG_PP_BLOCKS=$b timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/sq_$b -o run -- python3 scripts/vrun.py 16385 4 > gpurun_out/sq_$b.log 2>&1 || exit 1
done
python3 - <<'P'
import csv, glob, collections
for b in (3072, 512):
    f = glob.glob(f'gpurun_out/sq_{b}/**/run_counter_collection.csv', recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'k_postpre' in r['Kernel_Name']:
            acc[(r['Dispatch_Id'], r['Counter_Name'])].append(float(r['Counter_Value']))
    per = collections.defaultdict(list)
    for (d, c), v in acc.items(): per[c].append(sum(v))
    print(b, {c: round(sum(v)/len(v)) for c, v in sorted(per.items())})
P
