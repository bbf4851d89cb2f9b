set -o pipefail
O=gpurun_out/r02i; mkdir -p $O
RTRT_LIB=build/librtrt_ab.so timeout -k 10 200 python tools/ab.py --config b --env RTRT_HY_BLK --variants 22,11,21,41,42,44 --rounds 5 --frames 40 > $O/ab_blk_b.txt 2>&1 || exit $?
grep -o '"ms": {.*}}' $O/ab_blk_b.txt
