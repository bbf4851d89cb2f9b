# r03aa: per-frame PMC (FETCH/WRITE) and SQ counter runs for the batched configs a, b, c
# (--frame-batch 1: one frame per dispatch), then their bench lines with the counters attached
set -o pipefail
export TMPDIR=/tmp
T=r03aa; O=gpurun_out/$T; mkdir -p $O
export BENCH_ARGS="--frame-batch 1"
for c in b c a; do
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${c}_pmc_fetch -o run -- python3 bench.py --config $c --steps 3 --warmup 8 --no-cpu-baseline $BENCH_ARGS > /dev/null 2> $O/${c}_pmc_fetch.err || { tail $O/${c}_pmc_fetch.err; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${c}_pmc_write -o run -- python3 bench.py --config $c --steps 3 --warmup 8 --no-cpu-baseline $BENCH_ARGS > /dev/null 2> $O/${c}_pmc_write.err || { tail $O/${c}_pmc_write.err; exit 1; }
  python3 tools/pmc_summary.py $O/${c}_pmc_fetch $O/${c}_pmc_write $c $O/${c}_pmc.json || exit 1
  timeout -k 10 400 bash tools/pmc_config.sh $T $c kernel > $O/sq_${c}.txt 2>&1 || { tail $O/sq_${c}.txt; exit 1; }
  tail -2 $O/sq_${c}.txt
done
unset BENCH_ARGS
mkdir -p $O/prof
for c in b c a; do cp $O/${c}_pmc.json profiles/${T}_${c}_pmc.json; cp $O/sq_${c}.json profiles/${T}_sq_${c}.json; done
for c in b c a; do
  timeout -k 10 300 python -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail $O/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$c.json')); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['traffic'], r.get('valu_issue'), r.get('hardware_counters_note'))"
done
