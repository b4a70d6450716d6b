#!/bin/bash
# Runs tools/abl_probe.py once per environment setting ("A=1 B=2" per argument, "" = base);
# one JSON line each into gpurun_out/envsweep.jsonl.
set -o pipefail
mkdir -p gpurun_out
for e in "$@"; do
  env $e timeout -k 10 120 python -u tools/abl_probe.py 8 "${e:-base}" >> gpurun_out/envsweep.jsonl 2>> gpurun_out/envsweep.err || exit $?
  tail -n 1 gpurun_out/envsweep.jsonl
done
