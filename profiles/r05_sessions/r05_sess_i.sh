# r05 session i: kernel timelines of BASELINE configs[4]'s W call after the FMG start (32769)
# and of configs[1]'s 40-cycle call at 4097
set -u
export TMPDIR=/tmp
O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/g32769 -o run -- python3 scripts/cycle_timeline.py --child --kind G --n 32769 --cycles 1 > $O/g32769.log 2>&1 || exit $?
python3 scripts/cycle_timeline.py --parse $O/g32769 --kind G --cycles 1 > $O/tl_G32769.json || exit $?
rm -rf $O/g32769
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/v4097 -o run -- python3 scripts/cycle_timeline.py --child --whole --n 4097 --cycles 40 > $O/v4097.log 2>&1 || exit $?
python3 scripts/cycle_timeline.py --parse $O/v4097 --whole --cycles 40 > $O/tl_V4097_40.json || exit $?
rm -rf $O/v4097
