# Round-2 close-out measurement of the default kernel: GPU parity suite, smoke, bench lines
# (bench workload with the CPU baseline, configs[2] k_top 8/7 at 192 validators, configs[4]
# planted_deep), N=8 rank-share projection, drop-in time-to-verdict, rocprof stats + PMC.
# Outputs under gpurun_out/r02z/ and gpurun_out/prof_r02c/.
set -o pipefail
O=gpurun_out/r02d2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 2 --k-top 8 --validators 192 --no-cpu-baseline > $O/bench_192_k8.json 2> $O/bench_192_k8.err &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 2 --k-top 7 --validators 192 --no-cpu-baseline > $O/bench_192_k7.json 2> $O/bench_192_k7.err &&
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --workload planted_deep --no-cpu-baseline > $O/bench_planted_deep.json 2> $O/bench_planted_deep.err &&
timeout -k 10 200 python -u tools/rank_share_probe.py 8 2048 > $O/rank_share8.jsonl 2> $O/rank_share8.err &&
timeout -k 10 200 bash tools/ttv_cli.sh > $O/ttv_cli.log 2>&1 &&
bash tools/profile.sh r02d
rc=$?; tail -n 2 $O/gpu_tests.log; for f in bench_default bench_192_k8 bench_192_k7 bench_planted_deep; do python3 -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f',round(d['value']/1e9,2),round(d['ms_per_step'],3),d.get('golden','')[:5])" || true; done; tail -n 1 $O/rank_share8.jsonl | cut -c1-300; echo "exit $rc"; exit $rc
