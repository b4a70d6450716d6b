#!/bin/bash
# Collect the rocprofv3 evidence for bench.py's dominant kernel (run on the GPU box).
#   tools/profile.sh <tag> [bench args...]
# 1) kernel trace + stats; 2..n) PMC passes (one counter group per pass, no traces).
set -euo pipefail
TAG=${1:-r01}; shift || true
ARGS=${*:---steps 2 --warmup 1 --no-cpu-baseline}
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $ROOTDIR
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace_bench.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc1 -o run -- python3 bench.py $ARGS > $OUT/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc2 -o run -- python3 bench.py $ARGS > $OUT/pmc2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc3 -o run -- python3 bench.py $ARGS > $OUT/pmc3.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc4 -o run -- python3 bench.py $ARGS > $OUT/pmc4.log 2>&1
echo done > $OUT/DONE
