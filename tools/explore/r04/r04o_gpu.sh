# r04o: post-process blocks dealt to the XCDs as super-tiles of SX x SY blocks (4x4, 2x6, 4x12;
# variants built from a patched copy of the sources) against the in-tree mapping (runs of 4
# blocks along a row): per-launch time (same process), HBM bytes (PMC), pipelined frame
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04o; mkdir -p $O
L=real_time_ray_tracer_amd/librtrt.so,build/v_s4x4/librtrt.so,build/v_s2x6/librtrt.so,build/v_s4x12/librtrt.so
timeout -k 10 300 python -u tools/ab.py --config d --prog 2 --libs $L --rounds 6 --frames 10 --time-from 8 > $O/ab_post.txt 2>&1 || { tail -20 $O/ab_post.txt; exit 1; }
tail -1 $O/ab_post.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('post', {k: round(v['median'],4) for k,v in d['ms'].items()})"
for k in tree s4x4 s2x6 s4x12; do
  if [ $k = tree ]; then unset RTRT_LIB; else export RTRT_LIB=build/v_$k/librtrt.so; fi
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$k -o run -- python3 bench.py --config d --steps 10 --no-cpu-baseline > /dev/null 2> $O/pmc_fetch_$k.err
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$k -o run -- python3 bench.py --config d --steps 10 --no-cpu-baseline > /dev/null 2> $O/pmc_write_$k.err
  unset RTRT_LIB
  python3 tools/pmc_summary.py $O/pmc_fetch_$k $O/pmc_write_$k d $O/pmc_$k.json > /dev/null && python3 -c "import json; d=json.load(open('$O/pmc_$k.json')); print('$k post bytes', d['2'], round(d['2']/1592176622, 4))"
done
for i in 1 2 3; do
  for k in tree s4x4 s2x6 s4x12; do
    if [ $k = tree ]; then unset RTRT_LIB; else export RTRT_LIB=build/v_$k/librtrt.so; fi
    timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/d_${k}_$i.json 2> $O/d_${k}_$i.err || { tail $O/d_${k}_$i.err; exit 1; }
    unset RTRT_LIB
    python3 -c "import json; d=json.load(open('$O/d_${k}_$i.json')); print('d $k', $i, d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['kernel_ms'], d['roofline_post']['kernel_ms'])"
  done
done
