# Small grids for the first launches from the root (QI_SMALL_GRID): GPU suite, bench A/B,
# N=8 rank-share projection.  Outputs under gpurun_out/r02g/.
set -o pipefail
O=gpurun_out/r02g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -n 2 $O/gpu_tests.log
b() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$tag.json 2> $O/bench_$tag.err || return 1
  python3 -c "import json;d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]);print('$tag',round(d['value']/1e9,2),round(d['ms_per_step'],3),d['golden'][:5],d['roofline']['launches_per_step'],d['roofline']['avg_launch_ms'])"
}
for r in 1 2; do b full$r QI_SMALL_GRID=0 && b small$r QI_X=0 || exit 1; done
for g in 0 1; do
  QI_SMALL_GRID=$g timeout -k 10 200 python -u tools/rank_share_probe.py 8 2048 > $O/share_$g.jsonl 2> $O/share_$g.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/share_$g.jsonl').read().strip().splitlines()[-1]);print('share small=$g grow_ms',round(d['grow_ms'],3),'max_share',round(max(d['share_ms']),3),'est',round(d['est_step_ms'],3))"
done
