# strip overhead: mode 2 (AO pass alone) at config d, per-frame dispatch vs multi-frame launches
O=gpurun_out/r02z7; mkdir -p $O
timeout -k 10 250 python tools/strip_scaling.py --config d --n 8 --frames 24 --mode 2 > $O/m2_seq.txt 2>&1 || exit $?
timeout -k 10 250 python tools/strip_scaling.py --config d --n 8 --frames 24 --mode 2 --multi > $O/m2_multi.txt 2>&1 || exit $?
timeout -k 10 250 python tools/strip_scaling.py --config d --n 8 --frames 24 > $O/m1_pipe.txt 2>&1 || exit $?
tail -n 4 $O/m2_seq.txt $O/m2_multi.txt $O/m1_pipe.txt
