set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; tail -3 gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --cycle F --steps 10 --warmup 2 --cpu-baseline off --general-rhs off --pmc off > gpurun_out/benchF.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --cycle W --n 4097 --steps 3 --warmup 1 --cpu-baseline off --general-rhs off --pmc off > gpurun_out/benchW.log 2>&1 || exit 1
for f in bench benchF benchW; do python3 -c "
import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['unit'], d['ms_per_step'], d.get('parity'), d['roofline']['ms_per_launch'], d['roofline']['frac'], d['roofline'].get('traffic_ratio'))"; done
