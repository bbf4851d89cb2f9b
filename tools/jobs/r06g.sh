#!/usr/bin/env bash
# round 6 GPU job g: camera-relative sphere rows for the camera rays (build/v_camrel: Phong / hybrid;
# build/v_aocamrel: also the AO kernel's primary tests) against the previous build (build/v_prev)
set -uo pipefail
O=gpurun_out/r06g; mkdir -p $O
RTRT_LIB=build/v_camrel/librtrt.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_golden.py -m gpu -k "mode_parity or golden or moving or flying or camera or compute_frames" \
  > $O/tests_camrel.txt 2>&1
rc=$?; echo "rc=$rc" >> $O/tests_camrel.txt; tail -3 $O/tests_camrel.txt
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
RTRT_LIB=build/v_camrel/librtrt.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fullsize.py -m gpu -k "config_a or whole_frame and b-3 or tiles and (b-3 or s1)" > $O/tests_camrel_fullsize.txt 2>&1
echo "rc=$?" >> $O/tests_camrel_fullsize.txt; tail -3 $O/tests_camrel_fullsize.txt
for i in 1 2; do
  for v in prev camrel; do
    for c in b a; do
      RTRT_LIB=build/v_$v/librtrt.so timeout -k 10 120 python3 bench.py --config $c --no-cpu-baseline --no-alt-dispatch \
        > $O/${c}_${v}_$i.json 2> $O/${c}_${v}_$i.err || exit $?
      python3 -c "import json; d=json.loads(open('$O/${c}_${v}_$i.json').read().strip().splitlines()[-1]); print('$c', '$v', $i, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
    done
  done
done
RTRT_LIB=build/v_prev/librtrt.so timeout -k 10 300 python -u tools/ab.py --config d --libs build/v_prev/librtrt.so,build/v_aocamrel/librtrt.so \
  --rounds 4 --frames 4 > $O/ab_aocamrel_d.txt 2>&1 || exit $?
tail -1 $O/ab_aocamrel_d.txt | cut -c1-400
