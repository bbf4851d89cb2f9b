# r04k: bench lines + kernel traces for a, b (more frames), e, ref, p; GPU suite; smoke
set -o pipefail
bash tools/round_profile.sh bench r04j a b e ref p || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r04j/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r04j/gpu_tests.txt; exit 1; }; tail -3 gpurun_out/r04j/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04j/smoke.txt 2>&1; tail -2 gpurun_out/r04j/smoke.txt
