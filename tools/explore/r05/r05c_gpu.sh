#!/usr/bin/env bash
# round 5c: GPU suite on the correctly rounded sin build, SQ counters at (d), section clocks
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; tail -3 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
G1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -k 10 240 rocprofv3 --pmc $G1 --output-format csv -d $O/sq_d -o run -- python3 tools/ab.py --config d --variants 7 --rounds 1 --frames 2 > $O/sq_d.log 2>&1 || exit 1
RTRT_LIB=build/librtrt_ab.so timeout -k 10 240 python3 -u tools/sections.py --config d --variant 98 > $O/sections98_d.txt 2>&1 || exit 1
RTRT_LIB=build/librtrt_ab.so timeout -k 10 240 python3 -u tools/sections.py --config d --variant 97 > $O/sections97_d.txt 2>&1 || exit 1
cat $O/sections98_d.txt $O/sections97_d.txt
