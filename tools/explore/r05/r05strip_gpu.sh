#!/usr/bin/env bash
# round 5, last build: one-GPU strip-scaling estimates (each strip of an N-way split alone,
# calibrated plan, settled clocks) at (d) N = 8 and N = 4, and (e) N = 8
set -uo pipefail
O=gpurun_out/r05strip
mkdir -p $O
timeout -k 10 300 python3 -u tools/strip_scaling.py --config d --n 8 --calibrate --warm-ms 300 > $O/strip_scaling_d_n8_calibrated.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/strip_scaling.py --config d --n 4 --calibrate --warm-ms 300 > $O/strip_scaling_d_n4_calibrated.txt 2>&1 &&
timeout -k 10 500 python3 -u tools/strip_scaling.py --config e --n 8 --calibrate --warm-ms 300 --frames 4 > $O/strip_scaling_e_n8_calibrated.txt 2>&1
rc=$?
for f in $O/*.txt; do echo == $f; tail -4 $f; done
exit $rc
