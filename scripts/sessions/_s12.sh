set -o pipefail
mkdir -p gpurun_out/r02_final
export TMPDIR=/tmp
O=gpurun_out/r02_final
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off --general-rhs off --pmc off > $O/prof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --n 32769 --steps 5 --warmup 2 --cpu-baseline off --general-rhs off > $O/bench_32769.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --n 4097 --steps 20 --warmup 2 --cpu-baseline off --general-rhs off --pmc off > $O/bench_4097.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --cycle F --steps 10 --warmup 2 --cpu-baseline off --general-rhs off --pmc off > $O/bench_F.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --cycle W --n 4097 --steps 3 --warmup 1 --cpu-baseline off --general-rhs off --pmc off > $O/bench_W_4097.log 2>&1 || exit 1
PGMG_BENCH_SOLO=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 > $O/bench_solo2.log 2>&1 || exit 1
for f in bench bench_32769 bench_4097 bench_F bench_W_4097 bench_solo2; do python3 -c "
import json; d=json.loads([l for l in open('$O/$f.log') if l.startswith('{')][-1]); r=d['roofline']; print('$f', d['value'], d['unit'], d['ms_per_step'], d.get('parity'), r['ms_per_launch'], r['frac'], r.get('traffic_ratio'))"; done
