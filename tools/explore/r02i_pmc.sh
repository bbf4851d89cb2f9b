# PMC traffic + SQ counters + GPU suite + bench d for the final source (r02i: AB-only code removed, production kernels unchanged)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 8 --no-cpu-baseline --warm-ms 0 > /dev/null 2> $O/pmc_fetch.err || exit $?
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 3 --warmup 8 --no-cpu-baseline --warm-ms 0 > /dev/null 2> $O/pmc_write.err || exit $?
python3 tools/pmc_summary.py $O/pmc_fetch $O/pmc_write d $O/pmc.json || exit $?
timeout -k 10 300 tools/pmc_config.sh r02i d ao_batch > $O/pmc_sq_d.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('d',d['value'],d['ms_per_step'],d['ms_per_step_median'],r['kernel_ms'],r['frac'],r['traffic_on_this_build'])"
