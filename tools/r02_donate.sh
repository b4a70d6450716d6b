# Persistent-launch (QI_DONATE) check: smoke, bench A/B (kernel variants), GPU parity suite
# with donation on.  Outputs under gpurun_out/r02d/.
set -o pipefail
O=gpurun_out/r02d
mkdir -p $O
b() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$tag.json 2> $O/bench_$tag.err || return 1
  python3 -c "import json,sys;d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]);print('$tag',round(d['value']/1e9,2),round(d['ms_per_step'],3),d['golden'][:5],d['roofline']['launches_per_step'])"
}
QI_DONATE=1 timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
b on QI_DONATE=1 &&
b off QI_DONATE=0 &&
b base QI_DONATE=0 QI_JIT_DEFINES=QI_DONATE_CODE=0,QI_QMIN_ROUND=0 &&
b qmin QI_DONATE=0 QI_JIT_DEFINES=QI_DONATE_CODE=0 &&
b on2 QI_DONATE=1 QI_DQ_MARGIN=0 &&
b on3 QI_DONATE=1 QI_DQ_MARGIN=8192 QI_DQ_SHIFT=5 &&
QI_DONATE=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 3 $O/gpu_tests.log; echo "exit $rc"; exit $rc
