# Specialised kernel with per-SCC D-order LDS (8 waves/CU at SMAX 24) and smaller stacks
# for 9-10 waves/CU (QI_JIT_SMAX).  Outputs under gpurun_out/r02m/.
set -o pipefail
O=gpurun_out/r02m
mkdir -p $O
b() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$tag.json 2> $O/bench_$tag.err || return 1
  python3 -c "import json;d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]);print('$tag',round(d['value']/1e9,2),round(d['ms_per_step'],3),d['golden'][:5],d['roofline']['launches_per_step'],d['roofline']['units_per_step'])"
}
b s24 QI_X=0 && b s21 QI_JIT_SMAX=21 && b s18 QI_JIT_SMAX=18 && b s16 QI_JIT_SMAX=16 && b s24b QI_X=0 && b s21b QI_JIT_SMAX=21
