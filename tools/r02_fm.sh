# Removal-sensitivity minimality (QI_FASTMIN): GPU parity suite, then bench A/B + stamps.
set -o pipefail
O=gpurun_out/r02final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -n 2 $O/gpu_tests.log
b() {  # tag, defines
  QI_JIT_DEFINES="$2" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err || return 1
  python3 -c "import json;d=json.loads(open('$O/bench_$1.json').read().strip().splitlines()[-1]);print('$1',round(d['value']/1e9,2),round(d['ms_per_step'],3),d['golden'][:5],d['roofline']['launches_per_step'],d['roofline']['units_per_step'],d['roofline']['coop_phase_frac'])"
}
for r in 1 2; do b head$r "" || exit 1; done
timeout -k 10 120 python -u tools/stamps.py 10 > $O/stamps_fm.json 2>&1; grep -A8 cycles_per_iter $O/stamps_fm.json
