"""Candidates per target of the Model S neighbour passes against the z sub-cell count zsub (SPEC_SPH.md §0 row windows,
common.h row_window), on an interior block of the rest lattice (h = 1.2 dx, cells 2h): the pass-1 candidate cut finer
sub-cells could buy (verdict r5 item 4). CPU only.
    python scripts/zsub_candidates_model.py"""
import numpy as np
dx=0.01; h=1.2*dx; cell=2*h
rng=np.random.default_rng(1)
# interior block of a lattice
L=40
g=np.stack(np.meshgrid(*[np.arange(L)]*3,indexing='ij'),-1).reshape(-1,3)
pos=(g+0.5)*dx + rng.uniform(-1e-4,1e-4,g.shape)
# targets: interior ones
inner=np.all((g>12)&(g<L-12),1)
T=np.where(inner)[0][::37]
for zsub in (4,6,8,12,16):
    cz=cell/zsub
    cx=np.floor(pos[:,0]/cell).astype(int); cy=np.floor(pos[:,1]/cell).astype(int); czz=np.floor(pos[:,2]/cz).astype(int)
    # bucket
    from collections import defaultdict
    rows=defaultdict(list)
    for j,(a,b,c) in enumerate(zip(cx,cy,czz)): rows[(a,b)].append(j)
    rows={k:np.array(v) for k,v in rows.items()}
    cand=0; hits=0
    for t in T:
        p=pos[t]; fx=p[0]/cell-cx[t]; fy=p[1]/cell-cy[t]; gzf=p[2]/cz
        for ddx in (-1,0,1):
            for ddy in (-1,0,1):
                gx= fx if ddx<0 else (1-fx if ddx>0 else 0.0)
                gy= fy if ddy<0 else (1-fy if ddy>0 else 0.0)
                d2=gx*gx+gy*gy
                if d2>=1: continue
                hz=np.sqrt(1-d2)*zsub+1e-3
                zlo=int(max(gzf-hz,0)); zhi=int(gzf+hz)
                r=rows.get((cx[t]+ddx,cy[t]+ddy))
                if r is None: continue
                sel=r[(czz[r]>=zlo)&(czz[r]<=zhi)]
                cand+=len(sel)
                d=np.linalg.norm(pos[sel]-p,axis=1)
                hits+=np.sum(d<=2*h)
    print(zsub, "cand/target %.1f hits/target %.1f eff %.3f"%(cand/len(T),hits/len(T),hits/cand))
