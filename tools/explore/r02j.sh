set -o pipefail
O=gpurun_out/r02j; mkdir -p $O
RTRT_LIB=build/librtrt_ab.so timeout -k 10 200 python tools/ab.py --config b --env RTRT_HY_ABL --variants 0,5,1,3 --rounds 5 --frames 40 --allow-diff > $O/ab_abl_b.txt 2>&1 || exit $?
grep -o '"ms": {.*}}' $O/ab_abl_b.txt
