# Persistent-launch parity tests; ramp-budget A/B (bench + N=8 rank-share projection).
set -o pipefail
O=gpurun_out/r02r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k persistent -x -q --timeout 240 --timeout-method thread > $O/persistent_tests.log 2>&1 || { tail -30 $O/persistent_tests.log; exit 1; }
tail -n 2 $O/persistent_tests.log
b() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$tag.json 2> $O/bench_$tag.err || return 1
  python3 -c "import json;d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]);print('$tag',round(d['value']/1e9,2),round(d['ms_per_step'],3),d['golden'][:5],d['roofline']['launches_per_step'],d['roofline']['units_per_step'])"
}
s() {  # tag, per_rank, env...
  local tag=$1 pr=$2; shift 2
  env "$@" timeout -k 10 200 python -u tools/rank_share_probe.py 8 $pr > $O/share_$tag.jsonl 2> $O/share_$tag.err || return 1
  python3 -c "import json;d=json.loads(open('$O/share_$tag.jsonl').read().strip().splitlines()[-1]);print('share $tag grow_ms',round(d['grow_ms'],3),'max_share',round(max(d['share_ms']),3),'est',round(d['est_step_ms'],3),'seed',d['seed_units'])"
}
b r0 QI_X=0 && b r6 QI_RAMP_BUDGET=6 && b r12 QI_RAMP_BUDGET=12 && b r0b QI_X=0 && b r6b QI_RAMP_BUDGET=6 &&
s p2k 2048 && s p2k_r6 2048 QI_RAMP_BUDGET=6 && s p8k 8192 && s p8k_r6 8192 QI_RAMP_BUDGET=6 && s p16k_r6 16384 QI_RAMP_BUDGET=6
