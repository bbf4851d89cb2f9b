O=gpurun_out/r02ad; mkdir -p $O
export RTRT_LIB=build/librtrt_ab.so
# every workgroup renders the same pool (row 200 ground pool 120*... ): pool ids 48120 (row 200) and 240*1500+100
RTRT_POOL_ROT=0 RTRT_POOL_ILV=-48120 timeout -k 10 200 python tools/explore/xcd_balance.py one > $O/xcd_fix1.txt 2>&1 || exit $?
RTRT_POOL_ROT=0 RTRT_POOL_ILV=-360100 timeout -k 10 200 python tools/explore/xcd_balance.py one > $O/xcd_fix2.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/xcd_fix1.txt $O/xcd_fix2.txt | grep -v "block ->"
