#!/usr/bin/env python3
"""Why the exact_voxel_order mode is slow: the shape of libstdc++ introsort's partition phase on the
per-ring surf VoxelGrid keys of a C2 scan (the serial model of tests/test_voxel_order.py).

For each ring: its surf candidates (label <= 0 in the non-empty segments, featureExtraction.h:279-292),
their PCL voxel keys at odometrySurfLeafSize, then the partition phase level by level: levels until
every frame is <= 16, frames, and depth-exhausted frames (heap-sorted by std::partial_sort).
usage: ring_partition_depth.py
"""
import sys, numpy as np, collections
import os
R=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0,R); sys.path.insert(0,os.path.join(R,'oracle')); sys.path.insert(0,os.path.join(R,'tests'))
import pyoracle as O
from test_voxel_order import lg, median_to_first, partition
from feature_base_pointcloud_registration_amd import synth
P=synth.config_params("C2")
pts=synth.make_jobs("C2",1,base_seed=1000)[0][0]
pr=O.project(P,pts); f=O.Stream(P).features(pts)
cloud=pr["cloud"]; lab=f["label"]; sr=pr["start_ring"]; er=pr["end_ring"]
leaf=np.float32(P.odometry_surf_leaf_size); inv=np.float32(1.0)/leaf
stats=collections.Counter(); levels=[]; sizes=[]
def emulate_count(keys):
    n=len(keys); k=[int(x) for x in keys]; v=list(range(n))
    frames=[(0,n,2*lg(n))] if n>16 else []
    nlev=0; heap=0; heapn=0; nfr=0
    while frames:
        nlev+=1; nxt=[]
        for first,last,depth in frames:
            nfr+=1
            if depth==0: heap+=1; heapn+=last-first; continue
            depth-=1; mid=first+(last-first)//2
            median_to_first(k,v,first,first+1,mid,last-1)
            cut=partition(k,v,first+1,last,k[first])
            for ff in ((first,cut,depth),(cut,last,depth)):
                if ff[1]-ff[0]>16: nxt.append(ff)
        frames=nxt
    return nlev,heap,heapn,nfr
for r in range(64):
    s,e=sr[r],er[r]
    if e<=s: continue
    idx=[]
    for j in range(6):
        sp=(s*(6-j)+e*j)//6; ep=(s*(5-j)+e*(j+1))//6-1
        if sp<ep: idx+= [kk for kk in range(sp,ep+1) if lab[kk]<=0]
    c=cloud[idx]
    x=np.stack([c["x"],c["y"],c["z"]],1).astype(np.float32)
    mn=x.min(0); mx=x.max(0)
    mnb=np.floor(mn*inv).astype(np.int64); mxb=np.floor(mx*inv).astype(np.int64)
    dx=mxb-mnb+1
    ijk=np.floor(x*inv).astype(np.int64)-mnb
    keys=ijk[:,0]+ijk[:,1]*dx[0]+ijk[:,2]*dx[0]*dx[1]
    nlev,heap,heapn,nfr=emulate_count(keys)
    levels.append(nlev); sizes.append(len(keys)); stats['heap']+=heap; stats['heapn']+=heapn; stats['frames']+=nfr
print("rings",len(sizes),"mean n",np.mean(sizes),"levels mean/max",np.mean(levels),max(levels),dict(stats))
# per-level frames for ring 20
def levels_of(keys):
    n=len(keys); k=[int(x) for x in keys]; v=list(range(n))
    frames=[(0,n,2*lg(n))] if n>16 else []; out=[]
    while frames:
        out.append(sorted([l-f for f,l,d in frames],reverse=True)); nxt=[]
        for first,last,depth in frames:
            if depth==0: continue
            depth-=1; mid=first+(last-first)//2
            median_to_first(k,v,first,first+1,mid,last-1)
            cut=partition(k,v,first+1,last,k[first])
            for ff in ((first,cut,depth),(cut,last,depth)):
                if ff[1]-ff[0]>16: nxt.append(ff)
        frames=nxt
    return out
for r in (10,30):
    s,e=sr[r],er[r]; idx=[]
    for j in range(6):
        sp=(s*(6-j)+e*j)//6; ep=(s*(5-j)+e*(j+1))//6-1
        if sp<ep: idx+= [kk for kk in range(sp,ep+1) if lab[kk]<=0]
    c=cloud[idx]; x=np.stack([c["x"],c["y"],c["z"]],1).astype(np.float32)
    mnb=np.floor(x.min(0)*inv).astype(np.int64); mxb=np.floor(x.max(0)*inv).astype(np.int64); dx=mxb-mnb+1
    ijk=np.floor(x*inv).astype(np.int64)-mnb; keys=ijk[:,0]+ijk[:,1]*dx[0]+ijk[:,2]*dx[0]*dx[1]
    for L,fr in enumerate(levels_of(keys)): print(r, L, len(fr), fr[:8])
