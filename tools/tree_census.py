"""Census of the branch-and-bound tree of a tiered FBAS (k organisations of 3, inner 2-of-3,
outer ceil(2k/3)-of-k; pure Python, CPU): how many nodes are interior, leaves of which
kind, and which (exclusion child, inclusion child) class pairs interior nodes have.
Usage: python tools/tree_census.py 8    (k = 8: 1,857,737 nodes, ~1 min)"""
import sys
from collections import Counter
k=int(sys.argv[1]); m=3*k; thr=-(-2*k//3); half=m//2
orgs=[0b111<<(3*o) for o in range(k)]
pc=lambda x: bin(x).count('1')
def gfp(X):
    return X if sum(1 for o in orgs if pc(X&o)>=2)>=thr else 0
sys.setrecursionlimit(10000)
C=Counter(); nodes=0
# iterative DFS over (T,D,dlen)
stack=[(((1<<m)-1),0,0,'root')]
while stack:
    T,D,dlen,kind=stack.pop()
    nodes+=1
    if dlen>half or not (T|D): C[kind+':leaf0']+=1; continue
    if gfp(D): C[kind+':quorum']+=1; continue
    Q=gfp(T|D)
    if not Q or (D&~Q) or not (Q&~D): C[kind+':leaf']+=1; continue
    C[kind+':int']+=1
    c=Q&~D; b=(c&-c)
    Tn=c&~b
    # classify children for pair census
    def cls(T2,D2,dl,inc):
        if dl>half or not (T2|D2): return 'leaf0'
        if gfp(D2): return 'quorum'
        Q2=gfp(T2|D2)
        if not Q2 or (D2&~Q2) or not (Q2&~D2): return 'leaf'
        return 'int'
    C['pair e=%s i=%s'%(cls(Tn,D,dlen,0),cls(Tn,D|b,dlen+1,1))]+=1
    stack.append((Tn,D|b,dlen+1,'i'))
    stack.append((Tn,D,dlen,'e'))
print('nodes',nodes)
for k_,v in sorted(C.items()): print(k_,v, round(v/nodes,3))
