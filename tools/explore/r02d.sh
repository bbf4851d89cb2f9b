set -o pipefail
O=gpurun_out/r02d; mkdir -p $O
for c in p q; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
done
for c in d p q; do
  RTRT_LIB=build/librtrt_ab.so timeout -k 10 200 python tools/sections.py --config $c --frames 3 > $O/sections_$c.txt 2>&1 || exit $?
done
timeout -k 10 400 tools/pmc_config.sh r02d b hybrid > $O/pmc_b.txt 2>&1 || exit $?
cat $O/pmc_b.txt
