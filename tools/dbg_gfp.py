import sys, random
sys.path.insert(0,'tests'); sys.path.insert(0,'.')
from qi_testlib import *
import quorum_intersection_amd as qa
import numpy as np
for seed in (0, 2, 4):
    text = random_org_fbas(seed, 8)
    g = Oracle().load(text)
    f = qa.FBAS(text)
    rng = random.Random(seed)
    n=g.n
    nodes = random_masks(rng, n, 64, rng.uniform(0.3, 0.95))
    avail = [sorted(set(s) | {v for v in range(n) if rng.random() < 0.2}) for s in nodes]
    out = qa.sets_from_masks(f.gfp_batch(qa.masks_from_sets(nodes, n), qa.masks_from_sets(avail, n)), n)
    bad=0
    for i,(s,a,o) in enumerate(zip(nodes,avail,out)):
        av=[v in set(a) for v in range(n)]
        r=sorted(g.contains_quorum(s,av))
        if r!=o:
            bad+=1
            if bad<4: print(seed, i, 'oracle', r, 'gpu', o)
    print('seed', seed, 'n', n, 'bad', bad, 'of', len(nodes))
    # single query
    o1 = qa.sets_from_masks(f.gfp_batch(qa.masks_from_sets([list(range(n))], n), qa.masks_from_sets([list(range(n))], n)), n)
    print('all', o1, sorted(g.contains_quorum(list(range(n)), [True]*n)))
