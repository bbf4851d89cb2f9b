#!/usr/bin/env bash
# Run on the GPU box (via gpurun): bench + rocprofv3 kernel trace + separate PMC passes.
#   tools/profile_box.sh <tag> [config] [steps]
# Outputs under gpurun_out/<tag>/ (summaries to be copied into profiles/).
# BENCH_ARGS: extra bench.py arguments for the PMC passes (modes 2-4: "--frame-batch 1").
set -euo pipefail
TAG=${1:-r01}
CFG=${2:-d}
STEPS=${3:-20}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config "$CFG" --steps "$STEPS" --warmup 8 > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
  python3 bench.py --config "$CFG" --steps 10 --warmup 8 --no-cpu-baseline > "$OUT/kt_bench.json" 2> "$OUT/kt.err"
# the same bench sequential (--no-pipeline): every launch is a real kernel duration, so the
# rocprof --stats averages compare directly with the bench line's kernel_ms
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_seq" -o run -- \
  python3 bench.py --config "$CFG" --steps 10 --warmup 8 --no-cpu-baseline --no-pipeline > "$OUT/kt_seq_bench.json" 2> "$OUT/kt_seq.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
  python3 bench.py --config "$CFG" --steps 3 --warmup 8 --no-cpu-baseline ${BENCH_ARGS:-} > /dev/null 2> "$OUT/pmc_fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
  python3 bench.py --config "$CFG" --steps 3 --warmup 8 --no-cpu-baseline ${BENCH_ARGS:-} > /dev/null 2> "$OUT/pmc_write.err"
find "$OUT" -name "*.csv" | head -50
python3 tools/pmc_summary.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$CFG" "$OUT/pmc.json"
