# final build of round 2 (src 99249a856f8d): config d bench + rocprof kernel traces (pipelined and
# sequential) + PMC traffic, SQ counters of the AO kernel, so the bench line's traffic and VALU-issue
# fields are measured on this build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02q; mkdir -p $O
timeout -k 10 900 bash tools/profile_box.sh r02q d 20 > $O/profile_d.log 2>&1 || exit $?
timeout -k 10 300 tools/pmc_config.sh r02q d ao_batch > $O/pmc_sq_d.txt 2>&1 || exit $?
