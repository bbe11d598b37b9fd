# r05 session g: fp32 k_postpre_q4 -- the fp32 GPU tests, then an interleaved A/B against the
# 2-column build (libpgmg_base.so)
set -u
export TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -k "fp32 or f32" -x -q --timeout 200 --timeout-method thread > $O/tests_fp32.log 2>&1; rc=$?
echo "rc=$rc" >> $O/tests_fp32.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python -u scripts/pp_ab.py --dtype f32 --rounds 3 \
  base=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_base.so \
  q4=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg.so \
  q4b2048=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so:PGMG_PPQ_BLOCKS=2048 \
  q4b3072=parallel-geometric-multigrid-for-poisson-problem_amd/libpgmg_ab.so:PGMG_PPQ_BLOCKS=3072 > $O/pp_f32.jsonl 2> $O/pp_f32.err || exit $?
