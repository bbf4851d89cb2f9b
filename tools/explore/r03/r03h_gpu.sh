# r03h: where the AO kernel's wave time goes with / without the bounce-ray cluster cull (section clocks, variant 98)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03h; mkdir -p $O
export RTRT_LIB=build/librtrt_ab.so
for c in d c; do
  timeout -k 10 200 python -u tools/sections.py --config $c --variant 98 > $O/sections_${c}_clusters.txt 2>&1 || { tail $O/sections_${c}_clusters.txt; exit 1; }
  cat $O/sections_${c}_clusters.txt
  RTRT_NO_CLUSTERS=1 timeout -k 10 200 python -u tools/sections.py --config $c --variant 98 > $O/sections_${c}_noclusters.txt 2>&1 || { tail $O/sections_${c}_noclusters.txt; exit 1; }
  cat $O/sections_${c}_noclusters.txt
done
