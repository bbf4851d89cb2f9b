# round-2 profiles: config d full (bench + rocprof kernel trace, sequential trace, PMC), configs a/b/c/p bench +
# kernel trace, SQ counters on d and b, 8-way strip estimate
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02v; mkdir -p $O
timeout -k 10 900 bash tools/profile_box.sh r02v d 20 > $O/profile_d.log 2>&1 || exit $?
for c in a b c p; do
  timeout -k 10 300 python bench.py --config $c --steps $([ $c = a ] || [ $c = b ] && echo 400 || echo 20) > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$c -o run -- \
    python3 bench.py --config $c --steps $([ $c = a ] || [ $c = b ] && echo 80 || echo 10) --warmup 8 --no-cpu-baseline > $O/kt_bench_$c.json 2> $O/kt_$c.err || exit $?
done
timeout -k 10 300 tools/pmc_config.sh r02v d ao_batch > $O/pmc_sq_d.txt 2>&1 || exit $?
timeout -k 10 300 tools/pmc_config.sh r02v b hybrid > $O/pmc_sq_b.txt 2>&1 || exit $?
timeout -k 10 300 python tools/strip_scaling.py --config d --n 8 --frames 20 --calibrate > $O/strip_n8.txt 2>&1 || exit $?
tail -3 $O/strip_n8.txt
