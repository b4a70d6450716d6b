# HEAD check: GPU parity suite, smoke, default bench line.  Outputs under gpurun_out/r02h/.
set -o pipefail
mkdir -p gpurun_out/r02h
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02h/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02h/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 > gpurun_out/r02h/bench_default.json 2> gpurun_out/r02h/bench_default.err
rc=$?; tail -n 3 gpurun_out/r02h/gpu_tests.log; echo "exit $rc"; exit $rc
