#!/usr/bin/env bash
# kernel trace of one N-way strip rendered alone (pipelined), for the timeline tool
set -euo pipefail
N=${1:-8}; ONLY=${2:-3}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/strip_trace
mkdir -p "$OUT"; cd "$REPO"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o run -- \
  python3 tools/strip_scaling.py --config d --n "$N" --only "$ONLY" --frames 30 > "$OUT/log.txt" 2>&1
f=$(find "$OUT/kt" -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py "$f" 16 > "$OUT/timeline.txt"
python3 - "$f" > "$OUT/launches.txt" <<'PY'
import csv, sys
rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "ao_batch" in n or "post_kernel" in n:
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "AO" if "ao_" in n else "post", r.get("Queue_Id", ""), r.get("Stream_Id", "")))
rows.sort()
t0 = rows[0][0]
for s, e, k, q, st in rows[-40:]:
    print(f"{(s - t0) / 1e3:10.1f} us  {(e - s) / 1e3:8.1f} us  {k:4s} q={q} s={st}")
PY
