# Fast-step / full-iteration split (stamp set 4) for variants of the specialised kernel.
# Usage: bash tools/r03_st4.sh <tag> "<QI_JIT_DEFINES extra>" ...
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
i=0
for defs in "$@"; do
  QI_JIT_DEFINES=QI_STAMP_SET=4,QI_DIAG_FAST${defs:+,$defs} timeout -k 10 120 python -u tools/stamps.py 10 > $O/st4_$i.json 2> $O/st4_$i.err || exit 1
  python3 -c "
import json,sys;d=json.load(open('$O/st4_$i.json'));w=d['wave_iters'];f=d['coop_phases'];c=d['stamp_cycles']
print('$defs', 'iters',w,'fast',f,'full',w-f,'cyc/fast',round(c[0]/max(f,1)),'cyc/full',round(c[1]/max(w-f,1)),'total Gcyc',round((c[0]+c[1])/1e9,2),'kernel_ms',round(d['kernel_ms'],3),'launches',d['launches'])"
  i=$((i+1))
done
