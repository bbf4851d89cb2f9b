# r04p: the final build (d3fa69228d60): counters for every config, the driver's bench command,
# the GPU suite and smoke
set -o pipefail
bash tools/round_profile.sh counters r04p d b c a e ref p || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04p
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('driver bench', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline_post']['kernel_ms'], d['cpu_baseline']['value'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }; tail -3 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; tail -1 $O/smoke.txt
