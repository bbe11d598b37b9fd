set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fast.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/fast2.log 2>&1; rc=$?; grep -E "PASS|FAIL" gpurun_out/fast2.log; tail -2 gpurun_out/fast2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_fast.log 2>&1 || exit 1
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_fast.log') if l.startswith('{')][-1]); print(d['value'], d['parity'], d['roofline']['ms_per_launch'], d['roofline']['frac']); f=d['fast_mode']; print('FAST', f['value'], f['vs_exact'], f['roofline']['ms_per_launch'], f['roofline']['frac'], f['roofline']['traffic_ratio'])"
