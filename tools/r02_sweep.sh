# Grace / run_at re-sweep with the 128-iteration poll, interleaved twice.
set -o pipefail
O=gpurun_out/r02k4
mkdir -p $O
b() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$tag.json 2> $O/bench_$tag.err || return 1
  python3 -c "import json;d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]);print('$tag',round(d['value']/1e9,2),round(d['ms_per_step'],3),d['golden'][:5],d['roofline']['launches_per_step'],d['roofline']['units_per_step'])"
}
for r in 1 2; do
  b g24_$r QI_X=0 && b g16_$r QI_GRACE=16 && b g40_$r QI_GRACE=40 && b g64_$r QI_GRACE=64 && b ra3_$r QI_RUN_AT=3 && b ra5_$r QI_RUN_AT=5 || exit 1
done
