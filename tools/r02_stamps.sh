# Section breakdown (s_memtime stamps, jit=3 diagnostic build) of the search loop: the
# relaunch chain vs the persistent launch.  Outputs under gpurun_out/r02s/.
set -o pipefail
O=gpurun_out/r02s
mkdir -p $O
timeout -k 10 120 python -u tools/stamps.py 10 > $O/stamps_chain.json 2> $O/stamps_chain.err &&
QI_DONATE=1 timeout -k 10 120 python -u tools/stamps.py 10 > $O/stamps_donate.json 2> $O/stamps_donate.err
rc=$?; cat $O/stamps_chain.json $O/stamps_donate.json; exit $rc
