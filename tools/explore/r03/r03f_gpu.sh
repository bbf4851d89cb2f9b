# r03f: GPU suite; AO A/B old / clusters with pop_lowest survivors (in-tree) / with the streamed
# masked groups (build/stream) at d, c, e; post A/B old / planes / in-tree (XCD runs R = 5); PMC; bench d
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
L=build/old/librtrt.so,build/stream/librtrt.so,real_time_ray_tracer_amd/librtrt.so
for c in d c; do
timeout -k 10 300 python -u tools/ab.py --config $c --libs $L --rounds 5 --frames 6 --time-from 1 > $O/ab_ao_$c.txt 2>&1 || { tail -20 $O/ab_ao_$c.txt; exit 1; }
tail -1 $O/ab_ao_$c.txt
done
timeout -k 10 300 python -u tools/ab.py --config e --libs $L --rounds 2 --frames 3 --time-from 1 > $O/ab_ao_e.txt 2>&1 || { tail -20 $O/ab_ao_e.txt; exit 1; }
tail -1 $O/ab_ao_e.txt
timeout -k 10 300 python -u tools/ab.py --config d --libs build/old/librtrt.so,build/planes/librtrt.so,build/r4/librtrt.so,real_time_ray_tracer_amd/librtrt.so --prog 2 --rounds 5 --frames 12 --time-from 8 > $O/ab_post.txt 2>&1 || { tail -20 $O/ab_post.txt; exit 1; }
tail -1 $O/ab_post.txt
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --config d --steps 3 --warmup 8 --no-cpu-baseline > /dev/null 2> $O/pmc_fetch.err || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --config d --steps 3 --warmup 8 --no-cpu-baseline > /dev/null 2> $O/pmc_write.err || exit 1
python3 tools/pmc_summary.py $O/pmc_fetch $O/pmc_write d $O/pmc.json && cat $O/pmc.json
timeout -k 10 300 python -u bench.py --config d --steps 20 --warmup 8 --no-cpu-baseline > $O/bench_d.json 2> $O/bench_d.err && cat $O/bench_d.json
