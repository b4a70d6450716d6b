# Poll interval sweep on the round-2 kernel, interleaved; planted_deep (witness pruning
# through the polled best key) at the candidates.
set -o pipefail
O=gpurun_out/r02k3
mkdir -p $O
b() {  # tag, args, env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline $args > $O/bench_$tag.json 2> $O/bench_$tag.err || return 1
  python3 -c "import json;d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]);print('$tag',round(d['value']/1e9,2),round(d['ms_per_step'],3),d['golden'][:5],d['roofline']['launches_per_step'],d['roofline']['units_per_step'])"
}
for r in 1 2; do
  b p128_$r "" QI_JIT_DEFINES=QI_POLL_MASK=127 && b p256_$r "" QI_JIT_DEFINES=QI_POLL_MASK=255 && b p512_$r "" QI_JIT_DEFINES=QI_POLL_MASK=511 && b p1k_$r "" QI_JIT_DEFINES=QI_POLL_MASK=1023 || exit 1
done
b pd32 "--workload planted_deep" QI_X=0 && b pd128 "--workload planted_deep" QI_JIT_DEFINES=QI_POLL_MASK=127 && b pd512 "--workload planted_deep" QI_JIT_DEFINES=QI_POLL_MASK=511 &&
b k8_32 "--k-top 8 --validators 192" QI_X=0 && b k8_128 "--k-top 8 --validators 192" QI_JIT_DEFINES=QI_POLL_MASK=127 && b k8_512 "--k-top 8 --validators 192" QI_JIT_DEFINES=QI_POLL_MASK=511
