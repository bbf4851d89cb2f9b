# the driver's N=1 command on the final tree, twice
O=gpurun_out/r02j; mkdir -p $O
for k in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/b$k.json 2> $O/b$k.err || exit $?
  python3 -c "import json;d=json.load(open('$O/b$k.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],d['ms_per_step_median'],r['kernel_ms'],r['frac'],r['traffic_on_this_build'],(r.get('valu_issue') or {}).get('on_this_build'),d['cpu_baseline']['value'])"
done
