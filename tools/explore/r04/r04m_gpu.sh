# r04m: post-process blocks of 64 x (4 K) pixels, each wave K rows one after another (RT_POST_ROWS =
# K = 1, 4, 8): per-launch time (same process), HBM bytes (PMC), pipelined frame (alternating)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04m; mkdir -p $O
L=build/v_postrows1/librtrt.so,build/v_postrows4/librtrt.so,build/v_postrows8/librtrt.so
timeout -k 10 300 python -u tools/ab.py --config d --prog 2 --libs $L --rounds 6 --frames 10 --time-from 8 > $O/ab_post.txt 2>&1 || { tail -20 $O/ab_post.txt; exit 1; }
tail -1 $O/ab_post.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('post', {k: round(v['median'],4) for k,v in d['ms'].items()})"
for k in 1 4 8; do
  export RTRT_LIB=build/v_postrows$k/librtrt.so
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$k -o run -- python3 bench.py --config d --steps 10 --no-cpu-baseline > /dev/null 2> $O/pmc_fetch_$k.err
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$k -o run -- python3 bench.py --config d --steps 10 --no-cpu-baseline > /dev/null 2> $O/pmc_write_$k.err
  unset RTRT_LIB
  python3 tools/pmc_summary.py $O/pmc_fetch_$k $O/pmc_write_$k d $O/pmc_$k.json > /dev/null && python3 -c "import json; d=json.load(open('$O/pmc_$k.json')); print('rows $k post bytes', d['2'], round(d['2']/1592176622, 4))"
done
for i in 1 2 3; do
  for k in 1 4 8; do
    export RTRT_LIB=build/v_postrows$k/librtrt.so
    timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/d_rows${k}_$i.json 2> $O/d_rows${k}_$i.err || { tail $O/d_rows${k}_$i.err; exit 1; }
    unset RTRT_LIB
    python3 -c "import json; d=json.load(open('$O/d_rows${k}_$i.json')); print('d rows$k', $i, d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline_post']['kernel_ms'])"
  done
done
