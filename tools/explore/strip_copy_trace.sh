#!/usr/bin/env bash
# kernel + memory-copy trace of one N-way strip rendered alone (pipelined): when do the header
# copies and the AO / post launches of consecutive frames start and end
set -euo pipefail
N=${1:-8}; ONLY=${2:-3}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/strip_copy_trace
mkdir -p "$OUT"; cd "$REPO"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/kt" -o run -- \
  python3 tools/strip_scaling.py --config d --n "$N" --only "$ONLY" --frames 30 > "$OUT/log.txt" 2>&1
k=$(find "$OUT/kt" -name "*kernel_trace.csv" | head -1)
m=$(find "$OUT/kt" -name "*memory_copy_trace.csv" | head -1)
python3 - "$k" "$m" > "$OUT/events.txt" <<'PY'
import csv, sys
rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "ao_batch" in n or "post_kernel" in n:
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "AO" if "ao_" in n else "post", "q" + r.get("Queue_Id", "")))
if sys.argv[2]:
    for r in csv.DictReader(open(sys.argv[2])):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", "")[:12], "b" + r.get("Bytes", r.get("Size", ""))))
rows.sort()
t0 = rows[0][0]
for s, e, k, q in rows[-90:]:
    print(f"{(s - t0) / 1e3:10.1f} .. {(e - t0) / 1e3:10.1f} us  {k:18s} {q}")
PY
