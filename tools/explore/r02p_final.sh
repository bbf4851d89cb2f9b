# final tree of the round: GPU suite + smoke, the driver's N=1 bench command, config (a) bench + rocprof
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02p; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python bench.py --config a --steps 400 > $O/bench_a.json 2> $O/bench_a.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_a -o run -- \
  python3 bench.py --config a --steps 80 --warmup 8 --no-cpu-baseline > $O/kt_bench_a.json 2> $O/kt_a.err || exit $?
tail -c 300 $O/bench.json
