# r03j: GPU suite + AO A/B (old vs in-tree: bounce clusters in full and split-tail rounds, global
# split tails above 128 spheres) at d (8 rounds), c, e; bench lines for d and e
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
L=build/old/librtrt.so,real_time_ray_tracer_amd/librtrt.so
timeout -k 10 300 python -u tools/ab.py --config d --libs $L --rounds 8 --frames 6 --time-from 1 > $O/ab_ao_d.txt 2>&1 || { tail -20 $O/ab_ao_d.txt; exit 1; }
tail -1 $O/ab_ao_d.txt
timeout -k 10 300 python -u tools/ab.py --config c --libs $L --rounds 8 --frames 6 --time-from 1 > $O/ab_ao_c.txt 2>&1 || { tail -20 $O/ab_ao_c.txt; exit 1; }
tail -1 $O/ab_ao_c.txt
timeout -k 10 300 python -u tools/ab.py --config e --libs $L --rounds 2 --frames 3 --time-from 1 > $O/ab_ao_e.txt 2>&1 || { tail -20 $O/ab_ao_e.txt; exit 1; }
tail -1 $O/ab_ao_e.txt
timeout -k 10 300 python -u bench.py --config d --steps 20 --warmup 8 --no-cpu-baseline > $O/bench_d.json 2> $O/bench_d.err && cat $O/bench_d.json
timeout -k 10 400 python -u bench.py --config e --steps 4 --warmup 8 --no-cpu-baseline > $O/bench_e.json 2> $O/bench_e.err && cat $O/bench_e.json
