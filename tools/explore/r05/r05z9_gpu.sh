#!/usr/bin/env bash
# round 5z9: config (e) A/B of the cluster-mask build against the build before it (build/v_h5),
# then the whole GPU suite on the current build
set -uo pipefail
O=gpurun_out/r05z9
mkdir -p $O
L=build/v_h5/librtrt.so,real_time_ray_tracer_amd/librtrt.so
timeout -k 10 400 python -u tools/ab.py --config e --libs $L --rounds 2 --frames 2 > $O/ab_e.txt 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=5 > $O/gpu_tests.txt 2>&1
rc=$?
tail -1 $O/ab_e.txt | cut -c1-700; tail -3 $O/gpu_tests.txt
exit $rc
