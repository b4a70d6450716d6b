# Stochastic PC sampling of the bench's search kernel (instruction hot spots + stall
# reasons), then a kernel-trace timeline of the same command.  Run on the GPU box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pcs
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval 65536 --output-format csv -d $OUT/pc -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pc_bench.log 2>&1
echo "pc exit $?"
ls -R $OUT | head -30
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/trace_bench.log 2>&1
echo "trace exit $?"
