# round-2 final profiles (r02h): GPU suite + smoke, config d full (bench + rocprof kernel trace,
# sequential trace, PMC), configs a/b/c/p bench + kernel trace, SQ counters on d, N=4/8 strip estimates
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 900 bash tools/profile_box.sh r02h d 20 > $O/profile_d.log 2>&1 || exit $?
for c in a b c p; do
  timeout -k 10 300 python bench.py --config $c --steps $([ $c = a ] || [ $c = b ] && echo 400 || echo 20) > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$c -o run -- \
    python3 bench.py --config $c --steps $([ $c = a ] || [ $c = b ] && echo 80 || echo 10) --warmup 8 --no-cpu-baseline > $O/kt_bench_$c.json 2> $O/kt_$c.err || exit $?
done
timeout -k 10 300 tools/pmc_config.sh r02h d ao_batch > $O/pmc_sq_d.txt 2>&1 || exit $?
timeout -k 10 400 python tools/strip_scaling.py --config d --n 8 --frames 60 --warm-ms 300 --calibrate > $O/strip_n8.txt 2>&1 || exit $?
timeout -k 10 400 python tools/strip_scaling.py --config d --n 4 --frames 40 --warm-ms 300 --calibrate > $O/strip_n4.txt 2>&1 || exit $?
tail -n 1 $O/strip_n8.txt; tail -n 1 $O/strip_n4.txt
timeout -k 10 600 python tools/strip_scaling.py --config e --n 8 --frames 10 --warm-ms 300 --calibrate > $O/strip_e_n8.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --config e --steps 10 --warmup 8 --cpu-seconds 10 > $O/bench_e.json 2> $O/bench_e.err || exit $?
