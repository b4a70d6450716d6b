# Persistent-launch tuning: queue counters and bench lines for a few settings.
set -o pipefail
O=gpurun_out/r02q
mkdir -p $O
p() {  # tag, env...
  local tag=$1; shift
  env QI_DONATE=1 "$@" timeout -k 10 120 python -u tools/dq_probe.py 3 > $O/dq_$tag.jsonl 2> $O/dq_$tag.err || return 1
  echo "$tag $(tail -n 1 $O/dq_$tag.jsonl)"
}
p s7m1024 &&
p s5m1024 QI_DQ_SHIFT=5 &&
p s3m0 QI_DQ_SHIFT=3 QI_DQ_MARGIN=0 &&
p s3m8k QI_DQ_SHIFT=3 QI_DQ_MARGIN=8192
