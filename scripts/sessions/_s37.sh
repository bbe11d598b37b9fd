set -o pipefail
mkdir -p gpurun_out/r02_final6
export TMPDIR=/tmp
O=gpurun_out/r02_final6
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline off --general-rhs off --pmc off --other-configs off > $O/prof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --cycle W --n 4097 --steps 3 --warmup 1 --cpu-baseline off --general-rhs off --pmc off > $O/bench_W_4097.log 2>&1 || exit 1
python3 - <<'P'
import json
d=json.loads([l for l in open('gpurun_out/r02_final6/bench.log') if l.startswith('{')][-1])
r=d['roofline']; print('V', d['value'], d['parity'], r['ms_per_launch'], r['frac'], r['traffic_ratio'])
for o in d.get('other_configs', []): print(' ', {k: v for k, v in o.items() if k != 'config'})
print('gen', d['general_rhs']['value'], d['general_rhs']['roofline']['frac'])
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline_config1']['value'])
w=json.loads(open('gpurun_out/r02_final6/bench_W_4097.log').read().strip().splitlines()[-1]); print('W', w['value'])
f=d.get('fast_mode')
if f: print('FAST', f['value'], f['vs_exact'], f['roofline']['ms_per_launch'], f['roofline']['frac'])
P
