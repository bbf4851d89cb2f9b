# r04f: hybrid / Phong block order and LDS-table A/Bs (per-frame dispatch, configs b and a),
# alternating processes; post-process HBM bytes at (d) with the 64x4 tiles (PMC passes).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04f; mkdir -p $O
for i in 1 2 3; do
  for v in tree hyrev hynolds; do
    if [ $v = tree ]; then unset RTRT_LIB; else export RTRT_LIB=build/v_$v/librtrt.so; fi
    for c in b a; do
      timeout -k 10 200 python -u bench.py --config $c --steps 400 --no-cpu-baseline --no-alt-dispatch > $O/bench_${c}_${v}_$i.json 2> $O/bench_${c}_${v}_$i.err || { tail $O/bench_${c}_${v}_$i.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/bench_${c}_${v}_$i.json')); print('$c $v', $i, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
    done
  done
done
unset RTRT_LIB
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_d -o run -- python3 bench.py --config d --steps 10 --no-cpu-baseline > /dev/null 2> $O/pmc_fetch_d.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_d -o run -- python3 bench.py --config d --steps 10 --no-cpu-baseline > /dev/null 2> $O/pmc_write_d.err
python3 tools/pmc_summary.py $O/pmc_fetch_d $O/pmc_write_d d $O/pmc_d.json && cat $O/pmc_d.json
