# r05 session s: fp32 stencil stages as packed 2-vector arithmetic (PGMG_F32_PK): fp32 tests
# on the product build, then an interleaved A/B of the finest pass (scalar vs packed builds)
set -u
export TMPDIR=/tmp
O=gpurun_out/r05s; mkdir -p $O
P=$PWD/parallel-geometric-multigrid-for-poisson-problem_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp32.py tests/test_gpu_baseline_configs.py -q -x -k "fp32 or f32" --timeout 120 --timeout-method thread > $O/tests_f32.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/pp_ab.py --dtype f32 --rounds 3 pk0=$P/libpgmg_f32pk0.so pk1=$P/libpgmg_f32pk1.so > $O/ab_f32.jsonl 2> $O/ab_f32.err || exit $?
timeout -k 10 300 python -u scripts/pp_ab.py --dtype f32 --n 32769 --steps 10 --rounds 2 pk0=$P/libpgmg_f32pk0.so pk1=$P/libpgmg_f32pk1.so > $O/ab_f32_32769.jsonl 2>> $O/ab_f32.err || exit $?
timeout -k 10 300 python -u bench.py --dtype f32 --warmup 5 --steps 20 > $O/bench_f32.out 2> $O/bench_f32.err || exit $?
