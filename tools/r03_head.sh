# Round-3 HEAD check: GPU parity suite, smoke, default bench line.
set -o pipefail
O=gpurun_out/r03_head
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 > $O/bench_default.json 2> $O/bench_default.err
rc=$?; tail -n 2 $O/gpu_tests.log; cut -c1-600 $O/bench_default.json; echo "exit $rc"; exit $rc
