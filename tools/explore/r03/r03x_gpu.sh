# r03x: AO section clocks on the current build (A/B lib variants 98, 96, 97, 93) at config d
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03x; mkdir -p $O
for v in 98 96 97 93; do
RTRT_LIB=build/librtrt_ab.so timeout -k 10 200 python -u tools/sections.py --config d --variant $v > $O/sections_$v.txt 2>&1 || { tail $O/sections_$v.txt; exit 1; }
echo "== $v"; cat $O/sections_$v.txt | grep -v amdgpu.ids
done
