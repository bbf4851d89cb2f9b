#!/usr/bin/env bash
# The round's evidence set on the GPU box, for the library build in the tree:
#   tools/round_profile.sh <tag>
# GPU suite, smoke, the driver's bench command, rocprofv3 kernel traces (pipelined and sequential)
# with --stats, PMC FETCH_SIZE / WRITE_SIZE passes, SQ counter passes of the AO kernel (config d),
# settled-clock strip-scaling estimates (d: N = 4, 8; e: N = 8) and a gloo rehearsal of the N = 4
# launch (ranks sharing the GPU, gathered frames verified).  Outputs under gpurun_out/<tag>/.
set -o pipefail
TAG=${1:?tag}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 bash tools/profile_box.sh $TAG d 20 > $O/profile_box.txt 2>&1 || { tail -20 $O/profile_box.txt; exit 1; }
timeout -k 10 600 bash tools/pmc_config.sh $TAG d ao_batch > $O/sq_d.txt 2>&1 || { tail $O/sq_d.txt; exit 1; }
tail -2 $O/sq_d.txt
timeout -k 10 300 python -u tools/strip_scaling.py --config d --n 4 --frames 20 --calibrate --warm-ms 300 > $O/strip_scaling_n4_calibrated.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/strip_scaling.py --config d --n 8 --frames 20 --calibrate --warm-ms 300 > $O/strip_scaling_n8_calibrated.txt 2>&1 || exit 1
tail -3 $O/strip_scaling_n8_calibrated.txt
timeout -k 10 600 python -u tools/strip_scaling.py --config e --n 8 --frames 4 --calibrate --warm-ms 300 > $O/strip_scaling_e_n8_calibrated.txt 2>&1 || exit 1
tail -3 $O/strip_scaling_e_n8_calibrated.txt
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29537 bench.py --gpus 4 --backend gloo --steps 6 --warmup 8 --no-cpu-baseline > $O/gloo_n4.json 2> $O/gloo_n4.err || { tail -20 $O/gloo_n4.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/gloo_n4.json') if l.startswith('{')][-1]); print(d['value'], d['verify'], d['collective'], d['config']['strips'])"
