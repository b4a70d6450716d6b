# GPU parity suite + default bench line (no CPU baseline) into gpurun_out/$1/
set -o pipefail
O=gpurun_out/${1:-r03_check}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --workload planted_deep > $O/bench_deep.json 2> $O/bench_deep.err
rc=$?; tail -n 2 $O/gpu_tests.log; python3 - $O <<'PY'
import json,sys
for f in ("bench.json","bench_deep.json"):
    try:
        d=json.loads(open(sys.argv[1]+"/"+f).read().strip().splitlines()[-1])
        print(f, "ms", round(d["ms_per_step"],4), "frac", round(d["roofline"]["frac"],4), "launches", d["roofline"]["launches_per_step"], d["golden"])
    except Exception as e: print(f, "ERR", e)
PY
echo "exit $rc"; exit $rc
