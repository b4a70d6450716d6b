#!/bin/bash
# One GPU measurement round: bench (default config, 10 steps, no CPU leg), optionally the
# whole -m gpu suite.  Usage: bash tools/ab_run.sh <tag> [tests]   (extra env passes through)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || exit $?
python3 -c "import json,sys; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print('value', d['value']/1e9, 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], d['golden'])"
if [ "$2" = tests ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1; rc=$?
  tail -3 $out/tests.log
  exit $rc
fi
