"""Test support: a block-by-block CPU transliteration of nftree.hip's build
(big levels as rank pairings, small nodes depth first), used by the GPU
tests to localise a device-build difference to a level.  Not the oracle:
the tree itself is checked against oracle.tree (pinned to the reference's
nanoflann in test_nftree_cpu.py)."""
import numpy as np
T=8192; CH=2048; BT=256; PER=8; LEAF=100
f32=np.float32
def f2o(f):
    u=np.array([f],np.float32).view(np.uint32)[0]
    return int((~u)&0xffffffff) if u&0x80000000 else int(u|0x80000000)
def o2f(o):
    u=(o&0x7fffffff) if o&0x80000000 else ((~o)&0xffffffff)
    return np.array([u],np.uint32).view(np.float32)[0]
def nf_cut(t):
    EPS=f32(1e-5)
    max_span=f32(t['hi'][0]-t['lo'][0])
    for i in (1,2):
        sp=f32(t['hi'][i]-t['lo'][i])
        if sp>max_span: max_span=sp
    ms=f32(-1); cf=0
    for i in range(3):
        sp=f32(t['hi'][i]-t['lo'][i])
        if sp>f32(f32(1)-EPS)*max_span:
            spread=f32(o2f(t['mm'][3+i])-o2f(t['mm'][i]))
            if spread>ms: cf=i; ms=spread
    sv=f32(f32(t['lo'][cf]+t['hi'][cf])/f32(2))
    mn=o2f(t['mm'][cf]); mx=o2f(t['mm'][3+cf])
    cv = mn if sv<mn else (mx if sv>mx else sv)
    return cf, f32(cv)
def nf_index(c,l1,l2):
    if l1>c//2: return l1
    if l2<c//2: return l2
    return c//2
def build(P, stop=-1, trace=None, Lmax=None):
    n=len(P); vp=np.concatenate([P.astype(np.float32), np.arange(n)[:,None].astype(np.float32)],1)  # w as index (float ok here)
    idxs=np.arange(n)
    if Lmax is None:   # the device sizes its levels for a 16k-point bucket: pass its Lmax to compare stop by stop
        Lmax=0
        if n>T:
            l=0
            while (T<<l)<n: l+=1
            Lmax=min(l+9,40)
    nodes={}; nnodes=[1]
    lo=P.min(0).astype(np.float32); hi=P.max(0).astype(np.float32)
    pend={0:[dict(node=0,begin=0,count=n,lo=lo.copy(),hi=hi.copy(),mm=[f2o(lo[0]),f2o(lo[1]),f2o(lo[2]),f2o(hi[0]),f2o(hi[1]),f2o(hi[2])])]}
    small=[]; ntask={}
    for L in range(Lmax+1):
        if 0 <= stop <= L and L < Lmax:
            return vp[:,3].astype(np.int64)
        final = L>=Lmax
        np_ = 1 if L==0 else 2*ntask[L-1]
        Pl=pend.get(L,[])
        tasks=[]; ch=0
        for i in range(np_):
            e=Pl[i]
            valid=e['count']>0
            big= valid and not final and e['count']>T
            if big:
                e=dict(e); e['chunk0']=ch; e['nch']=(e['count']+CH-1)//CH; ch+=e['nch']; tasks.append(e)
            elif valid: small.append(dict(e))
        ntask[L]=0 if final else len(tasks)
        if trace is not None: trace.append((L, [dict(t) for t in tasks], len(small)))
        if final: break
        cmap=[]
        for t,tk in enumerate(tasks): cmap += [t]*tk['nch']
        pend[L+1]=[dict(count=0,mm=[0xffffffff]*3+[0]*3) for _ in range(2*len(tasks))]
        cA=[0]*ch; cAE=[0]*ch; cE2=[0]*ch
        # count
        for blk in range(ch):
            t=cmap[blk]; tk=tasks[t]; c=blk-tk['chunk0']
            feat,cut=nf_cut(tk)
            p0=c*CH; p1=min(p0+CH,tk['count'])
            x=vp[tk['begin']+p0:tk['begin']+p1,feat]
            cA[blk]=int((x<cut).sum()); cAE[blk]=int((x<=cut).sum())
            if c==0: tk['feat']=feat; tk['cut']=cut
        tblL=np.zeros_like(vp); tblR=np.zeros_like(vp)
        for PASS in (1,2):
            for TABLE in (True,False):
                newcE2=list(cE2)
                for blk in range(ch):
                    t=cmap[blk]; tk=tasks[t]; c=blk-tk['chunk0']; feat=tk['feat']; cut=tk['cut']
                    chunks=range(tk['chunk0'],tk['chunk0']+tk['nch'])
                    lim1=sum(cA[q] for q in chunks); before=sum(cA[q] for q in chunks if q<blk)
                    zlo,zhi=0,lim1
                    if PASS==2:
                        lim2=sum(cAE[q] for q in chunks); before=sum(cE2[q] for q in chunks if q<blk); zlo,zhi=lim1,lim2
                    ngood=zhi-zlo
                    p0=c*CH; p1=min(p0+CH,tk['count'])
                    seg=vp[tk['begin']+p0:tk['begin']+p1].copy()
                    good=(seg[:,feat]<cut) if PASS==1 else (seg[:,feat]==cut)
                    pref=before+np.concatenate([[0],np.cumsum(good)[:-1]])
                    ec=0
                    for j in range(len(seg)):
                        p=p0+j; out=seg[j]
                        if zlo<=p<zhi and not good[j]:
                            r=(p-zlo)-pref[j]
                            if TABLE: tblL[tk['begin']+r]=seg[j]
                            else: out=tblR[tk['begin']+r]
                        elif p>=zhi and good[j]:
                            r=ngood-pref[j]-1
                            if TABLE: tblR[tk['begin']+r]=seg[j]
                            else: out=tblL[tk['begin']+r]
                        if not TABLE:
                            vp[tk['begin']+p]=out
                            if PASS==1: ec+= out[feat]==cut
                    if not TABLE and PASS==1: newcE2[blk]=ec
                    if not TABLE and PASS==2:
                        index=nf_index(tk['count'],lim1,lim2)
                        for s in (0,1):
                            a,b=(p0,min(p1,index)) if s==0 else (max(p0,index),p1)
                            if b>a:
                                sl=vp[tk['begin']+a:tk['begin']+b,:3]
                                C=pend[L+1][2*t+s]
                                for q in range(3):
                                    C['mm'][q]=min(C['mm'][q],f2o(sl[:,q].min())); C['mm'][3+q]=max(C['mm'][3+q],f2o(sl[:,q].max()))
                        if c==0:
                            c1=nnodes[0]; nnodes[0]+=2
                            nodes[tk['node']]=(c1,c1+1,feat)
                            for s in (0,1):
                                C=pend[L+1][2*t+s]; C['node']=c1+s; C['begin']=tk['begin']+(0 if s==0 else index)
                                C['count']=index if s==0 else tk['count']-index
                                C['lo']=tk['lo'].copy(); C['hi']=tk['hi'].copy()
                                if s==0: C['hi'][feat]=cut
                                else: C['lo'][feat]=cut
                cE2=newcE2
    # small: DFS with rank pairing
    for tk in small:
        st=[(0,tk['count'],tk['node'],tk['lo'].copy(),tk['hi'].copy())]
        base=tk['begin']
        while st:
            lb,nn,node,lo,hi=st.pop()
            seg=vp[base+lb:base+lb+nn]
            mn=seg[:,:3].min(0); mx=seg[:,:3].max(0)
            if nn<=LEAF: nodes[node]=(base+lb,base+lb+nn,-1); continue
            t=dict(lo=lo,hi=hi,mm=[f2o(mn[0]),f2o(mn[1]),f2o(mn[2]),f2o(mx[0]),f2o(mx[1]),f2o(mx[2])])
            feat,cut=nf_cut(t)
            l1=int((seg[:,feat]<cut).sum()); l2=int((seg[:,feat]<=cut).sum())
            for (zlo,zhi,g) in ((0,l1,lambda a: a[:,feat]<cut),(l1,l2,lambda a: a[:,feat]==cut)):
                seg=vp[base+lb:base+lb+nn]; gg=g(seg)
                ML=[i for i in range(zlo,zhi) if not gg[i]]; MR=[i for i in range(nn-1,zhi-1,-1) if gg[i]]
                assert len(ML)==len(MR)
                a=seg[ML].copy(); bb=seg[MR].copy(); seg[ML]=bb; seg[MR]=a
                vp[base+lb:base+lb+nn]=seg
            index=nf_index(nn,l1,l2)
            c1=nnodes[0]; nnodes[0]+=2; nodes[node]=(c1,c1+1,feat)
            lo2=lo.copy(); hi2=hi.copy(); hi2[feat]=cut; lo3=lo.copy(); lo3[feat]=cut
            st.append((lb+index,nn-index,c1+1,lo3,hi.copy()))
            st.append((lb,index,c1,lo.copy(),hi2))
    return vp[:,3].astype(np.int64)
