# sections of the production AO kernel at config d: first bounce split (96) and event counts (97)
O=gpurun_out/r02z4; mkdir -p $O
export RTRT_LIB=build/librtrt_ab.so
timeout -k 10 200 python tools/sections.py --config d --variant 97 > $O/sec97_d.txt 2>&1 || exit $?
cat $O/sec96_d.txt $O/sec97_d.txt $O/sec93_d.txt | grep -v amdgpu.ids
