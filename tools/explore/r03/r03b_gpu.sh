set -o pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 600 python -u -m pytest tests/test_gpu_reference_instance.py tests/test_gpu_group.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r03b/tests.txt 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r03b/tests.txt; exit 1; }
tail -3 gpurun_out/r03b/tests.txt
timeout -k 10 300 python -u bench.py --config ref --steps 200 --warmup 10 > gpurun_out/r03b/bench_ref.json 2> gpurun_out/r03b/bench_ref.err || { echo BENCH REF FAILED; tail -20 gpurun_out/r03b/bench_ref.err; exit 1; }
cat gpurun_out/r03b/bench_ref.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 6 --warmup 8 --config c --no-cpu-baseline > gpurun_out/r03b/gloo_n2.json 2> gpurun_out/r03b/gloo_n2.err || { echo GLOO FAILED; tail -30 gpurun_out/r03b/gloo_n2.err; exit 1; }
cat gpurun_out/r03b/gloo_n2.json
