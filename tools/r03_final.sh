# Round-3 evidence run at the final kernel: GPU parity suite, smoke, default bench line with the
# complete CPU search timed in the same invocation, bench lines of the other configs,
# rank-share projections (N = 2, 4, 8; configs[3] and configs[4]), drop-in time-to-verdict,
# a 2-rank gloo rehearsal of bench.py's multi-process path on one GPU, section stamps, then
# rocprof stats + PMC passes.  Outputs under gpurun_out/r03f/ and gpurun_out/prof_r03/.
set -o pipefail
O=gpurun_out/r03f
mkdir -p $O
step() { echo "== $1" ; }
# the complete CPU search (~190 s on one core) prints nothing: keep a heartbeat in gpurun_out/
( while true; do sleep 45; date +%s >> $O/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step tests && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
step smoke && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
step bench_cpu_full && timeout -k 10 600 python -u bench.py --steps 20 --warmup 2 --cpu-full > $O/bench_default.json 2> $O/bench_default.err &&
step bench_driver_default && timeout -k 10 300 python -u bench.py > $O/bench_driver_default.json 2> $O/bench_driver_default.err &&
step bench_deep && timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --workload planted_deep > $O/bench_planted_deep.json 2> $O/bench_planted_deep.err &&
step bench_192 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --k-top 8 --validators 192 > $O/bench_192_k8.json 2> $O/bench_192_k8.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --k-top 7 --validators 192 > $O/bench_192_k7.json 2> $O/bench_192_k7.err &&
step shares && for w in 8 4 2; do timeout -k 10 250 python -u tools/rank_share_probe.py $w 2048 64 two_tier 2>> $O/share.err | tail -n 1 >> $O/rank_share_two_tier.jsonl || exit 1; done &&
timeout -k 10 250 python -u tools/rank_share_probe.py 8 2048 64 planted_deep 2>> $O/share.err | tail -n 1 >> $O/rank_share_planted_deep.jsonl &&
step shared_key && timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -s -k test_shared_best_key_prunes_other_engines --timeout 240 --timeout-method thread > $O/shared_best_key.log 2>&1 &&
step ttv && bash tools/ttv_cli.sh > $O/ttv_cli.log 2> $O/ttv_cli.err &&
step rehearse && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline > $O/rehearse2_gloo.log 2>&1 &&
step stamps && bash tools/r03_stamps.sh r03f > $O/stamps_summary.txt 2>&1 &&
step profile && bash tools/profile.sh r03
rc=$?; tail -n 2 $O/gpu_tests.log; cut -c1-300 $O/bench_default.json; cat $O/rank_share_two_tier.jsonl | cut -c1-200; echo "exit $rc"; exit $rc
