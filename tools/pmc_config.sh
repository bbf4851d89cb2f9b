#!/usr/bin/env bash
# SQ counter passes for one bench config (one rocprofv3 --pmc run per counter group, no
# tracing domains), summarised per kernel: tools/pmc_config.sh <tag> <config> [kernel-substring]
# BENCH_ARGS: extra bench.py arguments (modes 2-4: bench.py launches one frame per dispatch by default)
set -euo pipefail
TAG=$1
CFG=$2
KSUB=${3:-kernel}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$REPO"
export TMPDIR=/tmp
[ -f "$OUT/counters_list.txt" ] || timeout -k 5 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
G1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
G2="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
G3=${PMC_G3:-}
i=0
for G in "$G1" "$G2" $([ -n "$G3" ] && echo "G3"); do
  [ "$G" = "G3" ] && G="$G3"
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $G --output-format csv -d "$OUT/${CFG}_g$i" -o run -- \
    python3 bench.py --config "$CFG" --steps 10 --warmup 8 --no-cpu-baseline --no-alt-dispatch ${BENCH_ARGS:-} > "$OUT/${CFG}_g$i.log" 2>&1
done
python3 - "$OUT" "$CFG" "$KSUB" <<'EOF'
import csv, glob, os, sys, collections
out, cfg, ksub = sys.argv[1:4]
res = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sorted(glob.glob(os.path.join(out, f"{cfg}_g*"))):
    if not os.path.isdir(d):
        continue
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if ksub in k:
                name = k.replace("void ", "").replace("rt::(anonymous namespace)::", "").split("(rt::FrameParams")[0]
                res[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
import json
import shlex


def frames_per_dispatch(cfg, bench_args):
    """1 when every dispatch of the run renders one frame: mode 1 (the AO pass and the
    post-process launch per frame) always; modes 2-4 unless bench.py ran with --frame-batch > 1
    (its default, 1, is one launch per frame).  None: several frames per dispatch."""
    sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
    from bench import CONFIGS
    fb = 1
    a = shlex.split(bench_args)
    for i, x in enumerate(a):
        if x == "--frame-batch" and i + 1 < len(a):
            fb = int(a[i + 1])
        elif x.startswith("--frame-batch="):
            fb = int(x.split("=", 1)[1])
    return 1 if CONFIGS[cfg][4] == 1 or fb == 1 else None


try:  # the library build the counters were taken on (make lib writes BUILD_INFO)
    info = json.load(open(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "real_time_ray_tracer_amd", "BUILD_INFO")))
except Exception:
    info = {}
out_json = {"config": cfg, "kernels": {}, "src_sha1": info.get("src_sha1"), "commit": info.get("commit"),
            "units": "per dispatch, mean over the dispatches of the bench run (warm-up, timed, standalone, counted)",
            "bench_args": os.environ.get("BENCH_ARGS", ""),
            "frames_per_dispatch": frames_per_dispatch(cfg, os.environ.get("BENCH_ARGS", ""))}
for k, cs in res.items():
    avg = {c: round(sum(v) / len(v)) for c, v in sorted(cs.items())}
    print(cfg, k, avg, "dispatches", max(len(v) for v in cs.values()))
    out_json["kernels"][k] = avg
    out_json.setdefault("dispatches", {})[k] = max(len(v) for v in cs.values())
json.dump(out_json, open(os.path.join(out, f"sq_{cfg}.json"), "w"), indent=1)
EOF
