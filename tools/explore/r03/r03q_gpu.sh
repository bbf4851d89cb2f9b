# r03q: pipelined-frame floor without the post-process (A/B lib, RTRT_POST_SKIP=1) vs with it
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03q; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python -u tools/explore/pipeline_floor.py > $O/prod_$i.txt 2>&1 || { tail $O/prod_$i.txt; exit 1; }; echo prod $(cat $O/prod_$i.txt)
  RTRT_LIB=build/librtrt_ab.so timeout -k 10 200 python -u tools/explore/pipeline_floor.py > $O/ab_$i.txt 2>&1 || { tail $O/ab_$i.txt; exit 1; }; echo ab $(cat $O/ab_$i.txt)
  RTRT_LIB=build/librtrt_ab.so RTRT_POST_SKIP=1 timeout -k 10 200 python -u tools/explore/pipeline_floor.py > $O/skip_$i.txt 2>&1 || { tail $O/skip_$i.txt; exit 1; }; echo skip $(cat $O/skip_$i.txt)
done
RTRT_LIB=build/librtrt_ab.so RTRT_POST_SKIP=1 timeout -k 10 200 python -u tools/explore/pipeline_floor.py --no-pipeline > $O/skip_seq.txt 2>&1; echo skipseq $(cat $O/skip_seq.txt)
timeout -k 10 200 python -u tools/explore/pipeline_floor.py --no-pipeline > $O/prod_seq.txt 2>&1; echo prodseq $(cat $O/prod_seq.txt)
