"""Distinct fragment pairs among the LDS tail's records (numpy restatement of level 0 on R-MAT: two
Boruvka rounds, then the tail's rounds), per 256 consecutive-record blocks: how much a per-block
(da, db) minimum would shrink the records a tail round streams. A checker-side analysis (it uses
the oracle's R-MAT generator):  python tests/tools/tail_pairs.py 22"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import oracle as O
from scipy.sparse import coo_matrix
from scipy.sparse.csgraph import connected_components
sc=int(sys.argv[1])
n,u,v,w=O.rmat_canonical(sc)
u=np.asarray(u,np.int64);v=np.asarray(v,np.int64);w=np.asarray(w,np.int64); m=len(u)
eid=np.arange(m)
thr=np.sort(w)[int(0.45*n)]
L=w<thr
a=u[L]; b=v[L]; key=(w[L]<<32)|eid[L]
lab=np.arange(n)
def round_(a,b,key,lab):
    la=lab[a]; lb=lab[b]; live=la!=lb
    a,b,key,la,lb=a[live],b[live],key[live],la[live],lb[live]
    best=np.full(n,np.iinfo(np.int64).max)
    np.minimum.at(best,la,key); np.minimum.at(best,lb,key)
    win=(best[la]==key)|(best[lb]==key)
    g=coo_matrix((np.ones(win.sum()),(la[win],lb[win])),shape=(n,n))
    nc,comp=connected_components(g,directed=False)
    return a,b,key,comp[lab]
for r in range(2):
    a,b,key,lab=round_(a,b,key,lab)
    print('after round',r,'live',len(a))
la=lab[a]; lb=lab[b]; live=la!=lb
a,b,key,la,lb=a[live],b[live],key[live],la[live],lb[live]
print('tail records',len(a),'fragments',len(np.unique(np.concatenate([la,lb]))))
lo=np.minimum(la,lb); hi=np.maximum(la,lb)
pair=lo*n+hi
print('distinct pairs overall',len(np.unique(pair)))
G=256
Q=(len(pair)+G-1)//G
d=[len(np.unique(pair[i*Q:(i+1)*Q])) for i in range(G)]
print('per block records',Q,'distinct pairs per block: mean',np.mean(d),'max',max(d))
# next rounds in the tail
for r in range(3):
    best=np.full(n,np.iinfo(np.int64).max)
    np.minimum.at(best,la,key); np.minimum.at(best,lb,key)
    win=(best[la]==key)|(best[lb]==key)
    g=coo_matrix((np.ones(win.sum()),(la[win],lb[win])),shape=(n,n))
    nc,comp=connected_components(g,directed=False)
    la=comp[la]; lb=comp[lb]; live=la!=lb
    a,b,key,la,lb=a[live],b[live],key[live],la[live],lb[live]
    lo=np.minimum(la,lb); hi=np.maximum(la,lb); pair=lo*n+hi
    Q=(len(pair)+G-1)//G if len(pair) else 1
    d=[len(np.unique(pair[i*Q:(i+1)*Q])) for i in range(G)]
    print('tail round',r,'live',len(a),'frags',len(np.unique(np.concatenate([la,lb]))) if len(a) else 0,'pairs',len(np.unique(pair)),'per block mean',np.mean(d),'max',max(d))
