set -e
for wn in 0 9 17 33; do
  PGMG_TAIL_WAVE_N=$wn timeout -k 10 200 python bench.py --cycle W --n 4097 --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/bw_$wn.log 2>&1
  echo "wave_n=$wn $(tail -1 gpurun_out/bw_$wn.log | cut -c100-200)"
done
for wn in 0 17; do
  PGMG_TAIL_WAVE_N=$wn timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-baseline off > gpurun_out/bv_$wn.log 2>&1
  echo "V wave_n=$wn $(tail -1 gpurun_out/bv_$wn.log | cut -c100-200)"
done
