# Occupancy sensitivity of the specialised kernel: resident waves per CU (QI_JIT_WAVES).
set -o pipefail
O=gpurun_out/r02w
mkdir -p $O
for w in 7 6 5 4 7; do
  QI_JIT_WAVES=$w timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_w$w.json 2> $O/bench_w$w.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/bench_w$w.json').read().strip().splitlines()[-1]);print('waves/CU $w',round(d['value']/1e9,2),round(d['ms_per_step'],3),d['golden'][:5],d['roofline']['launches_per_step'])"
done
