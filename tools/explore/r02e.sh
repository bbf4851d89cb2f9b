set -o pipefail
O=gpurun_out/r02e; mkdir -p $O
for c in b a; do
  RTRT_LIB=build/librtrt_ab.so timeout -k 10 200 python tools/ab.py --config $c --env RTRT_TPB --variants 1,2,4,8 --rounds 3 --frames 40 > $O/ab_tpb_$c.txt 2>&1 || exit $?
  tail -1 $O/ab_tpb_$c.txt
done
