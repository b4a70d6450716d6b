# A/B of specialised-kernel variants (QI_JIT_DEFINES) on the bench workload, interleaved
# twice to expose box noise.  Outputs under gpurun_out/r02a/.
set -o pipefail
O=gpurun_out/r02a
mkdir -p $O
b() {  # tag, defines
  QI_JIT_DEFINES="$2" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err || return 1
  python3 -c "import json;d=json.loads(open('$O/bench_$1.json').read().strip().splitlines()[-1]);print('$1',round(d['value']/1e9,2),round(d['ms_per_step'],3),d['golden'][:5],d['roofline']['launches_per_step'],d['roofline']['units_per_step'])"
}
for r in 1 2; do
  b base$r "QI_EARLY_CLAIM=0,QI_REC_EARLY=0" && b early$r "QI_REC_EARLY=0" && b both$r "" || exit 1
done
