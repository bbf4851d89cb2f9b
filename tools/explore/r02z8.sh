O=gpurun_out/r02z8; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/clk -o run -- python3 tools/explore/clock_probe.py > $O/clk.log 2>&1 || exit $?
cat $O/clk.log | grep -v amdgpu.ids
find $O -name "*.csv" | head
python3 - $O <<'PY'
import csv, glob, sys
out = sys.argv[1]
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    print(f, len(rows), list(rows[0].keys()))
    for r in rows[:3]:
        print(r)
PY
