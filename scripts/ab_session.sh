set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/tests_cg.log 2>&1 || { tail -30 gpurun_out/tests_cg.log; exit 1; }
tail -2 gpurun_out/tests_cg.log
for v in t256 t512 default; do
  if [ $v = default ]; then L=""; else L=$PWD/scripts/libpgmg_$v.so; fi
  echo "== $v"
  PGMG_LIB=$L timeout -k 10 200 python bench.py --cycle W --n 4097 --steps 3 --warmup 1 --cpu-baseline off | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('W4097', d['value'], d['ms_per_step'])" || exit 1
  PGMG_CGRAPH_N=0 PGMG_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 2 --cpu-baseline off | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('V16385', d['value'], d['ms_per_step'])" || exit 1
done
for cg in 0 1025 2049 4097 8193; do
  for n in 16385 4097; do
   PGMG_CGRAPH_N=$cg timeout -k 10 200 python bench.py --n $n --steps 40 --warmup 3 --cpu-baseline off | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cg=$cg n=$n', d['value'], d['ms_per_step'])" || exit 1
  done
done
