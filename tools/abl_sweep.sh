#!/bin/bash
# Runs tools/abl_probe.py once per ablation (QI_JIT_DEFINES values, "" = base build);
# one JSON line each into gpurun_out/abl.jsonl.  Usage: bash tools/abl_sweep.sh "" "QI_ABL_NOREC" ...
set -o pipefail
mkdir -p gpurun_out
for d in "$@"; do
  QI_JIT_DEFINES="$d" timeout -k 10 120 python -u tools/abl_probe.py 8 "${d:-base}" >> gpurun_out/abl.jsonl 2>> gpurun_out/abl.err || exit $?
  tail -n 1 gpurun_out/abl.jsonl
done
