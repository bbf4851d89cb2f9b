# config (e) (the north star's 8-GPU config): one-GPU strip estimate at N=8 with settled clocks, and the N=1 bench
set -o pipefail
O=gpurun_out/r02bd; mkdir -p $O
timeout -k 10 600 python tools/strip_scaling.py --config e --n 8 --frames 10 --warm-ms 300 --calibrate > $O/strip_e_n8.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/strip_e_n8.txt
timeout -k 10 300 python bench.py --config e --steps 10 --warmup 8 --cpu-seconds 10 > $O/bench_e.json 2> $O/bench_e.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench_e.json'));r=d['roofline'];print('e',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],d['cpu_baseline'])"
