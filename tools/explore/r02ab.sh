O=gpurun_out/r02ab; mkdir -p $O
export RTRT_LIB=build/librtrt_ab.so
timeout -k 10 200 python tools/explore/xcd_balance.py > $O/xcd_rot.txt 2>&1 || exit $?
RTRT_POOL_ROT=0 timeout -k 10 200 python tools/explore/xcd_balance.py > $O/xcd_norot.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/xcd_rot.txt $O/xcd_norot.txt
