#!/usr/bin/env bash
# The round's evidence for the library build in the tree, on the GPU box:
#   tools/round_profile.sh counters <tag> <config>...   PMC FETCH_SIZE / WRITE_SIZE passes and the
#                                                       SQ counter passes per config (-> pmc_<c>.json,
#                                                       sq_<c>.json: copy them into profiles/ BEFORE
#                                                       the bench lines, which attach this build's)
#   tools/round_profile.sh bench <tag> <config>...      per config: the bench line with its CPU
#                                                       baseline, a rocprofv3 --kernel-trace --stats
#                                                       run of the same command, and the bench's
#                                                       kernel_ms against rocprof (tools/burst_check.py)
# Every GPU step has its own time limit; the script stops at the first failure.
set -eo pipefail
WHAT=${1:?counters|bench}; TAG=${2:?tag}; shift 2
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
ksub() { case $1 in a) echo phong_kernel;; b) echo hybrid_kernel;; *) echo ao_batch_kernel;; esac; }
for c in "$@"; do
  if [ "$WHAT" = counters ]; then
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$c -o run -- \
      python3 bench.py --config $c --steps 10 --no-cpu-baseline --no-alt-dispatch > /dev/null 2> $O/pmc_fetch_$c.err
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$c -o run -- \
      python3 bench.py --config $c --steps 10 --no-cpu-baseline --no-alt-dispatch > /dev/null 2> $O/pmc_write_$c.err
    python3 tools/pmc_summary.py $O/pmc_fetch_$c $O/pmc_write_$c $c $O/pmc_$c.json
    timeout -k 10 900 bash tools/pmc_config.sh $TAG $c $(ksub $c) > $O/sq_$c.txt 2>&1
    tail -3 $O/sq_$c.txt
  else
    timeout -k 10 600 python3 -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err
    python3 -c "import json,sys; d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['effective_frac'], d.get('cpu_baseline', {}).get('value'))"
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$c -o run -- \
      python3 bench.py --config $c --no-cpu-baseline > $O/kt_$c.json 2> $O/kt_$c.err
    python3 tools/burst_check.py $O/kt_$c/run_kernel_trace.csv $O/kt_$c.json > $O/burst_check_$c.txt
    cat $O/burst_check_$c.txt
  fi
done
