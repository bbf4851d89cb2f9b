# strip estimate with steady-state clocks (300 ms of frames before timing each case) vs without
O=gpurun_out/r02af; mkdir -p $O
timeout -k 10 400 python tools/strip_scaling.py --config d --n 8 --frames 60 --warm-ms 300 > $O/n8_warm.txt 2>&1 || exit $?
timeout -k 10 400 python tools/strip_scaling.py --config d --n 8 --frames 60 --warm-ms 300 --calibrate > $O/n8_warm_cal.txt 2>&1 || exit $?
tail -n 4 $O/n8_warm.txt $O/n8_warm_cal.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_d.json 2> $O/bench_d.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench_d.json'));print('d',d['value'],d['ms_per_step'],d['ms_per_step_median'],d['settle_frames'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
