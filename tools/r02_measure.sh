# Round-2 measurement session (one gpurun call): peaks, bench lines, CLI time-to-verdict,
# and the full CPU oracle run of the bench workload.  Outputs under gpurun_out/r02m/.
set -o pipefail
mkdir -p gpurun_out/r02m
timeout -k 10 60 ./tools/peak_probe > gpurun_out/r02m/peaks.json &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 > gpurun_out/r02m/bench_default.json 2> gpurun_out/r02m/bench_default.err &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 2 --k-top 8 --validators 192 --no-cpu-baseline > gpurun_out/r02m/bench_192_k8.json 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 2 --k-top 7 --validators 192 --no-cpu-baseline > gpurun_out/r02m/bench_192_k7.json 2>&1 &&
timeout -k 10 200 bash tools/ttv_cli.sh > gpurun_out/r02m/ttv_cli.log 2>&1 &&
timeout -k 10 400 taskset -c 0 python -u tools/cpu_full.py 10 256 > gpurun_out/r02m/cpu_full.json 2> gpurun_out/r02m/cpu_full.err
echo "exit $?"
