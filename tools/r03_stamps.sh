# Section breakdown (s_memtime stamps, jit=3 diagnostic build) of the search loop on the bench
# workload, one stamp set per run.  Outputs under gpurun_out/$1/.
set -o pipefail
O=gpurun_out/${1:-r03_stamps}
mkdir -p $O
for s in 4 0 1 2 3; do
  QI_JIT_DEFINES=QI_STAMP_SET=$s,QI_DIAG_FAST timeout -k 10 120 python -u tools/stamps.py 10 > $O/stamps_set$s.json 2> $O/stamps_set$s.err || exit $?
done
python3 - $O <<'PY'
import json,sys
for s in (4,0,1,2,3):
    d=json.load(open(f"{sys.argv[1]}/stamps_set{s}.json"))
    print(s, "wave_iters", d["wave_iters"], "fast", d["coop_phases"], "cyc/iter", round(d["cycles_per_wave_iter"]), "kernel_ms", round(d["kernel_ms"],3), d["cycles_per_iter"])
PY
