# r04h: AO pool schedule (longest first by wave time): its tests, the GPU suite, then (d)
# pipelined, (c) per frame and (b) with the schedule on / off and against the previous build
# (build/prev = af677b8: hybrid schedule only), alternating processes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_schedule.py -v -x --timeout 200 --timeout-method thread > $O/sched_tests.txt 2>&1 || { tail -40 $O/sched_tests.txt; exit 1; }; tail -7 $O/sched_tests.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }; tail -3 $O/gpu_tests.txt
run() {  # name, lib ('' = tree), args...
  local n=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export RTRT_LIB=$lib; else unset RTRT_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-alt-dispatch "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d.get('ms_per_step_median'), d['roofline']['kernel_ms'])"
  unset RTRT_LIB
}
for i in 1 2 3; do
  run d_prev_$i build/prev/librtrt.so --steps 40 --warmup 5
  run d_on_$i "" --steps 40 --warmup 5
  run d_off_$i "" --steps 40 --warmup 5 --no-tile-schedule
  run c_prev_$i build/prev/librtrt.so --config c --steps 60
  run c_on_$i "" --config c --steps 60
  run c_off_$i "" --config c --steps 60 --no-tile-schedule
  run b_on_$i "" --config b --steps 800
  run b_off_$i "" --config b --steps 800 --no-tile-schedule
done
