# r03i: GPU suite (in-tree: clusters in full rounds with 4-survivor loads + split tails); AO A/B old /
# clusters full rounds only, one-at-a-time survivors (tg0) / in-tree / + global-table split tails above 128 spheres (gt)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
L=build/old/librtrt.so,build/tg0/librtrt.so,real_time_ray_tracer_amd/librtrt.so,build/gt/librtrt.so
for c in d c; do
timeout -k 10 300 python -u tools/ab.py --config $c --libs $L --rounds 5 --frames 6 --time-from 1 > $O/ab_ao_$c.txt 2>&1 || { tail -20 $O/ab_ao_$c.txt; exit 1; }
tail -1 $O/ab_ao_$c.txt
done
timeout -k 10 300 python -u tools/ab.py --config e --libs $L --rounds 2 --frames 3 --time-from 1 > $O/ab_ao_e.txt 2>&1 || { tail -20 $O/ab_ao_e.txt; exit 1; }
tail -1 $O/ab_ao_e.txt
