#!/bin/bash
# Tuning sweep on the GPU box: one bench.py line per configuration (no CPU baseline).
#   tools/sweep.sh "<ENV=.. args>" "<ENV=.. args>" ...
# Each argument is "VAR=val ... -- bench args"; results go to gpurun_out/sweep.jsonl.
set -uo pipefail
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOTDIR"
mkdir -p gpurun_out
OUT=gpurun_out/sweep.jsonl
: > $OUT
for cfg in "$@"; do
  envs=${cfg%%--*}
  args=${cfg#*--}
  [ "$envs" == "$cfg" ] && args=""
  line=$(env $envs timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps ${SWEEP_STEPS:-60} --warmup 5 $args 2>gpurun_out/sweep_err.log | grep '"metric"')
  rc=$?
  if [ $rc -ne 0 ]; then echo "{\"cfg\": \"$cfg\", \"rc\": $rc}" >> $OUT; tail -n 20 gpurun_out/sweep_err.log; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(sys.argv[2]); r=d['roofline']; print(json.dumps({'cfg': sys.argv[1], 'value': d['value'], 'ms': d['ms_per_step'], 'avg_launch_ms': r['avg_launch_ms'], 'launches': r['launches_per_step'], 'occ': r['lane_occupancy'], 'coop': r['coop_phase_frac'], 'units': r['units_per_step']}))" "$cfg" "$line" >> $OUT
  tail -n 1 $OUT
done
