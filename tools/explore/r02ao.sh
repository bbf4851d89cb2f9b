# split depth planes: GPU suite, bench d (post kernel time), PMC bytes of the post-process
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02ao; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_d.json 2> $O/bench_d.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench_d.json'));r=d['roofline'];p=d['roofline_post'];print('d',d['value'],d['ms_per_step'],d['ms_per_step_median'],r['kernel_ms'],r['frac'],'post',p['kernel_ms'],p['frac'])"
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 8 --no-cpu-baseline --warm-ms 0 > /dev/null 2> $O/pmc_fetch.err || exit $?
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 3 --warmup 8 --no-cpu-baseline --warm-ms 0 > /dev/null 2> $O/pmc_write.err || exit $?
python3 tools/pmc_summary.py $O/pmc_fetch $O/pmc_write d $O/pmc.json && cat $O/pmc.json
