# Stack layout / depth / grid A/B in one box (twice).  Outputs under gpurun_out/r02o/.
set -o pipefail
O=gpurun_out/r02o
mkdir -p $O
b() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$tag.json 2> $O/bench_$tag.err || return 1
  python3 -c "import json;d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]);print('$tag',round(d['value']/1e9,2),round(d['ms_per_step'],3),d['golden'][:5],d['roofline']['launches_per_step'],d['roofline']['units_per_step'])"
}
for r in 1 2; do
b pk32s24_$r QI_JIT_DEFINES=QI_PK16=0 && b pk16s24w9_$r QI_X=0 && b pk16s24w8_$r QI_JIT_WAVES=8 && b pk16s28_$r QI_JIT_SMAX=28 || exit 1
done
