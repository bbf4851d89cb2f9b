set -e
for i in 1 2 3; do
  RTRT_LIB=build/old/librtrt.so timeout -k 10 200 python tools/ab.py --config d --variants 7 --rounds 2 --frames 4 2>&1 | grep "round 1" | sed "s/^/old /"
  timeout -k 10 200 python tools/ab.py --config d --variants 7 --rounds 2 --frames 4 2>&1 | grep "round 1" | sed "s/^/new /"
done
