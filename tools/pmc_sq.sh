#!/usr/bin/env bash
# SQ counter passes (one rocprofv3 --pmc run per counter group, no tracing domains) for the
# trace kernel under each AO variant.  Usage: tools/pmc_sq.sh <tag> <variants...>
set -euo pipefail
TAG=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
G1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
G2="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for v in "$@"; do
  i=0
  for G in "$G1" "$G2"; do
    i=$((i+1))
    RTRT_AO_VARIANT=$v timeout -k 10 240 rocprofv3 --pmc $G --output-format csv -d "$OUT/v${v}_g$i" -o run -- \
      python3 tools/ab.py --config d --variants "$v" --rounds 1 --frames 2 > "$OUT/v${v}_g$i.log" 2>&1
  done
done
python3 - "$OUT" <<'EOF'
import csv, glob, os, sys, collections
out = sys.argv[1]
for d in sorted(glob.glob(os.path.join(out, "v*_g*"))):
    if not os.path.isdir(d): continue
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "ao_" in r["Kernel_Name"] and "kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(d), {k: round(sum(v) / len(v)) for k, v in agg.items()})
EOF
