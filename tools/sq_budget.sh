#!/usr/bin/env bash
# Instruction budget of the production AO kernel at (d): SQ_INSTS_VALU / SALU / LDS / SMEM per
# launch of the A/B library's copies of the production instantiation, alone (101) and with one
# section's work repeated once (102 cluster-round tests, 103 culled primary tests, 104 the five
# hashes, 105 first-bounce survivor iterations; round 6: 106 the hit shading's arithmetic, 107 the
# primary setup after the hashes, 108 the hand-out shuffles, 109 the first bounce's cone + cull,
# 110 the full rounds' cluster cull): each difference is that section's instructions.
#   tools/sq_budget.sh <tag>     (on the GPU box; make ablib first)
set -euo pipefail
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
G="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
for v in ${VARIANTS:-101 102 103 104 105 106 107 108 109 110}; do
  RTRT_LIB=build/librtrt_ab.so RTRT_AO_VARIANT=$v timeout -s KILL 180 rocprofv3 --pmc $G --output-format csv \
    -d $O/v$v -o run -- python3 tools/ab.py --config d --variants $v --rounds 1 --frames 2 --allow-diff > $O/v$v.log 2>&1
done
python3 - "$O" <<'PY'
import csv, glob, os, sys, collections, json
out = sys.argv[1]
res = {}
for d in sorted(glob.glob(os.path.join(out, "v1??"))):
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "ao_batch_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    res[os.path.basename(d)] = {k: sum(v) / len(v) for k, v in agg.items()}
base = res.get("v101", {})
names = {"v102": "cluster-round survivor tests", "v103": "culled primary tests", "v104": "five hashes (binary64 sin)",
         "v105": "first-bounce survivor iterations", "v106": "hit shading arithmetic (every segment)",
         "v107": "primary setup after the hashes", "v108": "hand-out shuffles (13 per hand-out)",
         "v109": "first-bounce cone + per-sphere cull", "v110": "full rounds' cluster cull"}
print(json.dumps({"per_launch": res}, indent=1))
for v, n in names.items():
    if v in res and base:
        d = {k: res[v][k] - base[k] for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS")}
        print(f"{n:36s} VALU {d['SQ_INSTS_VALU']/1e6:8.1f} M ({100*d['SQ_INSTS_VALU']/base['SQ_INSTS_VALU']:5.1f}%)  "
              f"SALU {d['SQ_INSTS_SALU']/1e6:8.1f} M ({100*d['SQ_INSTS_SALU']/base['SQ_INSTS_SALU']:5.1f}%)  "
              f"LDS {d['SQ_INSTS_LDS']/1e6:6.1f} M")
print(f"{'total (production)':36s} VALU {base.get('SQ_INSTS_VALU',0)/1e6:8.1f} M  SALU {base.get('SQ_INSTS_SALU',0)/1e6:8.1f} M")
PY
