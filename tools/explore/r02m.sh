for v in 7; do RTRT_HY_ABL=$v RTRT_LIB=build/librtrt_ab.so timeout -k 10 120 python tools/explore/wave_timeline.py b 2>&1 | grep -v amdgpu.ids; done
