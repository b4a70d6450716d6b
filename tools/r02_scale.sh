# Scaling / launch-shape experiments on one GPU (rank_share_probe emulates an N-rank split).
set -o pipefail
mkdir -p gpurun_out/scale
timeout -k 10 200 python -u tools/stamps.py > gpurun_out/scale/stamps.json 2>&1 || exit 1
for cfg in "X=0 -- 8 2048" "QI_MID_BUDGET=256 -- 8 2048" "QI_MID_BUDGET=64 -- 8 2048" "QI_RUN_AT=8 -- 8 2048" "X=0 -- 8 8192" "QI_MID_BUDGET=64 -- 8 8192" "X=0 -- 4 2048" "X=0 -- 2 2048"; do
  envs=${cfg%%--*}; args=${cfg#*--}
  echo "== $cfg" >> gpurun_out/scale/probe.log
  env $envs timeout -k 10 120 python -u tools/rank_share_probe.py $args >> gpurun_out/scale/probe.log 2>&1 || exit 1
done
for cfg in "X=0" "QI_MID_BUDGET=256" "QI_MID_BUDGET=64"; do
  echo "== $cfg" >> gpurun_out/scale/bench.log
  env $cfg timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline >> gpurun_out/scale/bench.log 2>&1 || exit 1
done
echo done
