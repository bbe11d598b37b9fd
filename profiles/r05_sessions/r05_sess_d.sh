set -u
export TMPDIR=/tmp
O=gpurun_out/r05d; mkdir -p $O
L=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/tests.log
case $rc in 124|134|137|139) exit $rc;; esac
PGMG_LIB=$L/libpgmg_ab.so timeout -k 10 300 python -u scripts/op_ip_ab.py --rounds 2 > $O/op_ip_ab.jsonl 2> $O/op_ip_ab.err || exit $?
for v in base new; do
  if [ $v = base ]; then export PGMG_LIB=$L/libpgmg_base.so; else export PGMG_LIB=$L/libpgmg.so; fi
  timeout -k 10 300 python bench.py --dtype f32 --warmup 2 --steps 20 --cpu-baseline off --pmc off --ops off --dropin off > $O/bench_f32_$v.json 2> $O/bench_f32_$v.err || exit $?
done
unset PGMG_LIB
