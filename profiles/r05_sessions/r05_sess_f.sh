# r05 session f: coarse-end timelines (16385, 4097), per-rank strip compute at 16385 and 32769
# (W = 1, 2, 4, 8, SOLO ranks), and a kernel trace of the op study's in-place Jacobi calls
set -u
export TMPDIR=/tmp
O=gpurun_out/r05f; mkdir -p $O
bash scripts/coarse_session.sh $O/coarse > $O/coarse.log 2>&1 || exit $?
timeout -k 10 400 python3 scripts/strip_probe.py --n 32769 --steps 10 > $O/strip_probe_32769.jsonl 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/opprof -o run -- python3 scripts/op_ip_ab.py --quick --rounds 1 > $O/opprof.log 2>&1 || exit $?
