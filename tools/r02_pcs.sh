# Default-kernel bench and persistent-launch queue counters.  (PC sampling is refused on
# this pool: kernel traces and PMC counters only.)
set -o pipefail
O=gpurun_out/r02p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err &&
QI_DONATE=1 timeout -k 10 120 python -u tools/dq_probe.py 3 > $O/dq_probe.jsonl 2> $O/dq_probe.err
rc=$?; echo "exit $rc"; cat $O/dq_probe.jsonl; ls -R $O | head -30; exit $rc
