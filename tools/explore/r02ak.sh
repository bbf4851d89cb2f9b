# moving-camera parity tests (small sizes, all modes; config d tiles at 4K)
set -o pipefail
O=gpurun_out/r02ak; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k moving -v --timeout 300 --timeout-method thread > $O/moving.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/moving.log | tail -15; exit $rc
