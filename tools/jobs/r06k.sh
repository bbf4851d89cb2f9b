#!/usr/bin/env bash
# round 6 GPU job k: the camera / shadow survivor loops with the next survivor's rows requested
# before the current test (build/v_campf, -DRT_CAM_PF=1) against production (build/v_base)
set -uo pipefail
O=gpurun_out/r06k; mkdir -p $O
RTRT_LIB=build/v_campf/librtrt.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_adversarial.py -m gpu -k "mode_parity or golden or moving or adversarial" \
  > $O/tests_campf.txt 2>&1
rc=$?; echo "rc=$rc" >> $O/tests_campf.txt; tail -2 $O/tests_campf.txt
[ $rc -ne 0 ] && exit $rc
RTRT_LIB=build/v_campf/librtrt.so timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fullsize.py -m gpu -k "config_a or whole_frame and b-3" > $O/tests_campf_fullsize.txt 2>&1
rc=$?; echo "rc=$rc" >> $O/tests_campf_fullsize.txt; tail -2 $O/tests_campf_fullsize.txt
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do for v in base campf; do for c in b a; do
  RTRT_LIB=build/v_$v/librtrt.so timeout -k 10 120 python3 bench.py --config $c --no-cpu-baseline --no-alt-dispatch \
    > $O/${c}_${v}_$i.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.loads(open('$O/${c}_${v}_$i.json').read().strip().splitlines()[-1]); print('$c', '$v', $i, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done; done; done
