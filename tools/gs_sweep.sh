# Sweep of experimental kernel knobs on the bench workload (run on the GPU box).
set -o pipefail
cd $GRAFT_REPO_ROOT
W=${W:-two_tier}
run() { echo "== $*"; env "$@" timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $BARGS > gpurun_out/gs.log 2>&1 || { tail -5 gpurun_out/gs.log; exit 1; }; tail -n 1 gpurun_out/gs.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value']/1e9,2), 'Gev/s', round(d['ms_per_step'],3),'ms', 'launches', r['launches_per_step'], 'occ', round(r['lane_occupancy'],3), 'coop', round(r['coop_phase_frac'],3), 'avg_ms', round(r['avg_launch_ms'],4))"; }
for v in "$@"; do run $v; done
