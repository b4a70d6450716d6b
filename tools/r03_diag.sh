# Per-launch wave phase times (QI_DIAG_LAUNCH build) of one bench search and of one N=8 share.
set -o pipefail
O=gpurun_out/${1:-r03_diag}
mkdir -p $O
export QI_JIT_DEFINES=QI_DIAG_LAUNCH${2:+,$2}
timeout -k 10 120 python -u tools/launch_trace.py > $O/n1.log 2>&1 &&
timeout -k 10 120 python -u tools/share_trace.py 8 2048 0 > $O/share8.log 2>&1
rc=$?; grep "launch\|step:" $O/n1.log | cut -c1-330; echo; grep "launch\|step:\|====" $O/share8.log | tail -16 | cut -c1-330; exit $rc
