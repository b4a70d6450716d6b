# Persistent-launch tuning: queue counters for a few settings, then a donate-on bench line.
set -o pipefail
O=gpurun_out/r02q
mkdir -p $O
p() {  # tag, env...
  local tag=$1; shift
  env QI_DONATE=1 "$@" timeout -k 10 120 python -u tools/dq_probe.py 3 > $O/dq_$tag.jsonl 2> $O/dq_$tag.err || return 1
  echo "$tag $(tail -n 1 $O/dq_$tag.jsonl)"
}
p m0 QI_DQ_MARGIN=0 &&
p m1024 &&
p m8k QI_DQ_MARGIN=8192 &&
QI_DONATE=1 timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_on.json 2> $O/bench_on.err &&
python3 -c "import json;d=json.loads(open('$O/bench_on.json').read().strip().splitlines()[-1]);print('bench on',round(d['value']/1e9,2),round(d['ms_per_step'],3),d['golden'][:5])"
