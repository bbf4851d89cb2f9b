O=gpurun_out/r02ae; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU --kernel-trace --output-format csv -d $O/clk -o run -- python3 tools/explore/clock_probe.py > $O/clk.log 2>&1 || exit $?
grep "ms/frame" $O/clk.log
python3 - $O <<'PY'
import csv, glob, sys
out = sys.argv[1]
f = glob.glob(out + "/**/*counter_collection.csv", recursive=True)[0]
d = {}
for r in csv.DictReader(open(f)):
    if 'ao_batch' not in r['Kernel_Name']: continue
    e = d.setdefault(int(r['Dispatch_Id']), {'grid': int(r['Grid_Size']), 'dur': (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3})
    e[r['Counter_Name']] = float(r['Counter_Value'])
for k in sorted(d):
    e = d[k]
    clk = e['GRBM_GUI_ACTIVE'] / 8 / e['dur'] / 1e3
    occ = e['SQ_WAVE_CYCLES'] * 4 / (e['dur'] * 1e3 * clk) / 1024  # waves per SIMD (quad-cycles)
    print(k, e['grid'], f"{e['dur']:.0f} us clk {clk:.3f} waves/SIMD {occ:.2f} valu/wave {e['SQ_INSTS_VALU'] / e['SQ_WAVES']:.0f} waves {e['SQ_WAVES']:.0f}")
PY
