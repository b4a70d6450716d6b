# Two-rank rehearsal of bench.py's multi-process path on one GPU (gloo), plus the driver's
# default bench invocation and smoke.  Outputs under gpurun_out/r02e/.
set -o pipefail
O=gpurun_out/r02e
mkdir -p $O
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench_driver_default.json 2> $O/bench_driver_default.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline > $O/rehearse2.log 2>&1
rc=$?; tail -n 2 $O/smoke.log; python3 -c "import json;d=json.loads(open('$O/bench_driver_default.json').read().strip().splitlines()[-1]);print('default',round(d['value']/1e9,2),d['ms_per_step'],d['golden'][:5])"; grep -h '"metric"' $O/rehearse2.log | cut -c1-260; echo "exit $rc"; exit $rc
