set -o pipefail
O=gpurun_out/r02_lvl
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -n 2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -n 20 $O/bench.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); r=d['roofline']
print('V', d['value'], d['parity'], r['ms_per_launch'], r['frac'], r.get('traffic_ratio'))"
timeout -k 10 700 python scripts/level_pmc.py run --out $O/levels > $O/levels.jsonl 2>&1; rc=$?; cut -c1-400 $O/levels.jsonl; exit $rc
