# Round-2 measurement of the default kernel: GPU parity suite, smoke, bench line (with the
# CPU baseline), N=8 rank-share projection (relaunch chain and persistent launches), then
# the rocprof stats + PMC passes.  Outputs under gpurun_out/r02f/ and gpurun_out/prof_r02b/.
set -o pipefail
O=gpurun_out/r02f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 200 python -u tools/rank_share_probe.py 8 2048 > $O/share8.jsonl 2> $O/share8.err &&
QI_DONATE=1 timeout -k 10 200 python -u tools/rank_share_probe.py 8 2048 > $O/share8_donate.jsonl 2> $O/share8_donate.err &&
bash tools/profile.sh r02b
rc=$?; tail -n 2 $O/gpu_tests.log; tail -n 1 $O/share8.jsonl | cut -c1-400; tail -n 1 $O/share8_donate.jsonl | cut -c1-400; echo "exit $rc"; exit $rc
