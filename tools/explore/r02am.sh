# A/B: first-bounce pre-test for scenes above the LDS sphere-table size (RTRT_PT_BIG), config e;
# parity of that path on the scene-size tests
set -o pipefail
O=gpurun_out/r02am; mkdir -p $O
export RTRT_LIB=build/librtrt_ab.so
RTRT_PT_BIG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "scene_sizes or spp_variants" -q --timeout 200 --timeout-method thread > $O/tests_ptbig.log 2>&1; rc=$?
tail -2 $O/tests_ptbig.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab.py --config e --env RTRT_PT_BIG --variants 0,1 --rounds 2 --frames 3 > $O/e.txt 2>&1 || exit $?
grep -h "round\|^{" $O/e.txt | grep -v counters
