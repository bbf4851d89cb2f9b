# r04i: AO waves per CU limited through its LDS allocation (24 / 26 per CU instead of 28) so a
# post-process wave fits beside them in the pipelined frame; (d), alternating processes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04i; mkdir -p $O
run() {  # name, lib ('' = tree), args...
  local n=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export RTRT_LIB=$lib; else unset RTRT_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-alt-dispatch "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d.get('ms_per_step_median'), d['roofline']['kernel_ms'], d['roofline_post']['kernel_ms'])"
  unset RTRT_LIB
}
for i in 1 2 3; do
  run d_tree_$i "" --steps 40 --warmup 5
  run d_lds6800_$i build/v_aolds6800/librtrt.so --steps 40 --warmup 5
  run d_lds6300_$i build/v_aolds6300/librtrt.so --steps 40 --warmup 5
done
