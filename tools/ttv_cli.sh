# Time-to-verdict through the drop-in executable (stdin open -> verdict printed), device
# init apart (QI_TIMING), with a cold and a warm run-time-specialisation cache.
#   bash tools/ttv_cli.sh > gpurun_out/ttv_cli.log
set -e
python3 -c "import sys; sys.path.insert(0,'.'); from quorum_intersection_amd import fbas_gen; open('gpurun_out/two_tier_10_256.json','w').write(fbas_gen.two_tier(10,256)); open('gpurun_out/two_tier_8_192.json','w').write(fbas_gen.two_tier(8,192)); open('gpurun_out/planted_deep_8_512.json','w').write(fbas_gen.planted_deep(8,512))"
cache=$(mktemp -d)
for w in two_tier_10_256 two_tier_8_192 planted_deep_8_512; do
  rm -rf "$cache"; mkdir -p "$cache"
  for run in cold warm warm; do
    t_start=$(date +%s.%N)
    out=$(QI_JIT_CACHE="$cache" QI_TIMING=1 timeout -k 5 60 ./bin/quorum_intersection < gpurun_out/$w.json 2>gpurun_out/ttv_err.txt || true)
    t_end=$(date +%s.%N)
    # process_wall_ms: the whole process, exit status included (a cold run compiles the
    # specialised kernel after printing the verdict)
    echo "{\"workload\": \"$w\", \"cache\": \"$run\", \"verdict\": \"$out\", \"process_wall_ms\": $(python3 -c "print(round(($t_end - $t_start) * 1e3, 1))"), \"timing\": $(tail -n1 gpurun_out/ttv_err.txt)}"
  done
done
