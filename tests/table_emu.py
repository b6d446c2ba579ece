"""Pure-Python restatement of the device smoother's run-space algorithm
(csrc/h3d_table.hip k_disp_table: points as runs of copies, windows by
binary search, the delta-skipping schedule as a next-fit chain, weighted
order statistics for the median). Test infrastructure: tests/test_table_emu.py
holds it bit-equal to the host smoother (h3d_disp_table, itself pinned to the
reference's tables) on random and golden columns, which is what licenses the
reformulation; the GPU tests then hold the kernel bit-equal to the host."""
import bisect
import math

import numpy as np

def rolling_var(v):
    n=len(v); w=20; off=(w-1)//2
    out=[math.nan]*n
    st=[min(max(i+1+off-w,0),n) for i in range(n)]; en=[min(max(i+1+off,0),n) for i in range(n)]
    S=dict(mean=0.,ss=0.,nobs=0.,ca=0.,cr=0.,prev=0.,consec=0)
    def add(val):
        if val!=val: return
        S['nobs']+=1
        S['consec'] = S['consec']+1 if val==S['prev'] else 1
        S['prev']=val
        pm=S['mean']-S['ca']; y=val-S['ca']; t=y-S['mean']; S['ca']=t+S['mean']-y
        S['mean']=S['mean']+t/S['nobs'] if S['nobs'] else 0.
        S['ss']=S['ss']+(val-pm)*(val-S['mean'])
    def rem(val):
        if val==val:
            S['nobs']-=1
            if S['nobs']:
                pm=S['mean']-S['cr']; y=val-S['cr']; t=y-S['mean']; S['cr']=t+S['mean']-y
                S['mean']=S['mean']-t/S['nobs']; S['ss']=S['ss']-(val-pm)*(val-S['mean'])
            else: S['mean']=0.; S['ss']=0.
    for i in range(n):
        if i==0 or st[i]>=en[i-1]:
            S.update(prev=v[st[i]],consec=0,mean=0.,ss=0.,nobs=0.,ca=0.,cr=0.)
            for j in range(st[i],en[i]): add(v[j])
        else:
            for j in range(st[i-1],st[i]): rem(v[j])
            for j in range(en[i-1],en[i]): add(v[j])
        if S['nobs']>=w and S['nobs']>1:
            out[i]=0. if (S['nobs']==1 or S['consec']>=S['nobs']) else S['ss']/(S['nobs']-1.)
    return out

def pairwise(a):
    n=len(a)
    if n<8:
        r=0.
        for x in a: r+=x
        return r
    if n<=128:
        r=list(a[:8]); i=8
        while i < n-(n%8):
            for j in range(8): r[j]+=a[i+j]
            i+=8
        res=((r[0]+r[1])+(r[2]+r[3]))+((r[4]+r[5])+(r[6]+r[7]))
        for x in a[i:]: res+=x
        return res
    n2=n//2; n2-=n2%8
    return pairwise(a[:n2])+pairwise(a[n2:])

def interp(xp, yp, xn):
    m=len(xp); idx=bisect.bisect_left(xp,xn); idx=min(max(idx,1),m-1)
    slope=(yp[idx]-yp[idx-1])/(xp[idx]-xp[idx-1])
    return slope*(xn-xp[idx-1])+yp[idx-1]

def emu(col, weighted=True, frac=-1., aff=15.):
    D=len(col)
    X=[float(d) for d in range(D) if math.isfinite(col[d])]; Y=[col[d] for d in range(D) if math.isfinite(col[d])]
    n0=len(X)
    if n0<2: return 'fail'
    lb=Y[0]; inc=0
    if weighted:
        var=rolling_var(Y)
        WT=[]
        for v in var:
            prec = 1.0/v if v!=0 else (math.inf if v==v else math.nan)
            if v!=v: prec=math.nan
            WT.append(math.pow(prec,0.25) if math.isfinite(prec) else math.nan)
        fin=[w for w in WT if w==w]
        if not fin: return 'fail'
        min_w=min(fin); inv=1.0/min_w
        SW=[(1.0 if w==min_w else w*inv) for w in WT]
        max_w=max([s for s in SW if s==s])
        SW=[max_w if (s==math.inf or s==-math.inf) else s for s in SW]
        ff=next((i for i,s in enumerate(SW) if math.isfinite(s)), n0)
        left_w=SW[ff if ff<n0 else 0]
        for i in range(n0):
            if SW[i]!=SW[i]:
                if i < n0/2.0: SW[i]=left_w
                elif i > n0/2.0: SW[i]=1.
            if not math.isfinite(SW[i]): return 'fail'
        fi=next((i for i in range(n0-1) if Y[i+1]-Y[i]>0), n0)
        inc=(fi if fi<n0 else 0)+1
        if not (frac>=0):
            nm=pairwise(fin)/len(fin)
            frac=max(min(aff/(max_w*nm),2./3),0.05)
        runs=[(X[i],Y[i],int(math.floor(SW[i]))) for i in range(inc,n0) if math.floor(SW[i])>=1]
    else:
        if not (frac>=0): frac=0.3
        runs=[(X[i],Y[i],1) for i in range(n0)]
    U=len(runs); RX=[r[0] for r in runs]; RY=[r[1] for r in runs]; CNT=[r[2] for r in runs]
    RP=[0]
    for c in CNT: RP.append(RP[-1]+c)
    n=RP[-1]
    if n<2 or U<2: return 'fail'
    k=int(frac*n+1e-10); k=min(max(k,2),n)
    delta=(RX[-1]-RX[0])*0.01
    def run_of(p): return bisect.bisect_right(RP,p)-1
    LEFT=[0]*U; NXT=[0]*U
    for u in range(U):
        xval=RX[u]; lo,hi=0,n-k
        while lo<hi:
            mid=(lo+hi)//2
            if xval > (RX[run_of(mid)]+RX[run_of(mid+k)])/2.0: lo=mid+1
            else: hi=mid
        LEFT[u]=lo
        cut=xval+delta
        a=u+1
        while a<U and not RX[a]>cut: a+=1
        if a<U: NXT[u]= a-1 if a-1>u else u+1
        elif u==U-1: NXT[u]=-1
        else: NXT[u]=run_of(max(n-2,RP[u+1]))
    FL=[]; u=0
    while True:
        FL.append(u)
        if u==U-1 or NXT[u]<0: break
        u=NXT[u]
    br=[bisect.bisect_right(FL,u)-1 for u in range(U)]
    RW=[1.]*U; FIT=[0.]*U
    for rob in range(4):
        for u in FL:
            xval=RX[u]; left=LEFT[u]; right=left+k
            r0=run_of(left); r1=run_of(right-1)
            radius=max(xval-RX[r0], RX[r1]-xval); ir=1.0/radius
            S0=S1=S2=T0=T1=0.
            for r in range(r0,r1+1):
                cc=float(min(RP[r+1],right)-max(RP[r],left)); d=RX[r]-xval
                t=abs(d)*ir; uu=1-t*(t*t); uu=uu if uu>0 else 0.; wt=uu*(uu*uu)
                if rob>0: wt=wt*RW[r]
                cw=cc*wt; cwd=cw*d
                S0+=cw; S1+=cwd; S2+=cwd*d; T0+=cw*RY[r]; T1+=cwd*RY[r]
            if S0<=0: f=RY[u]
            else:
                iv=1.0/S0; m=S1*iv; t0=T0*iv; var=S2*iv-m*m; f=t0-m*(T1*iv-m*t0)/var
            FIT[u]=f
        for u in range(U):
            j=br[u]
            if FL[j]!=u:
                ua,ub=FL[j],FL[j+1]; a=(RX[u]-RX[ua])/(RX[ub]-RX[ua]); FIT[u]=a*FIT[ub]+(1.0-a)*FIT[ua]
        if not all(math.isfinite(f) for f in FIT): return 'degenerate'
        if rob==3: break
        AB=[abs(RY[u]-FIT[u]) for u in range(U)]
        pts=sorted(sum([[AB[u]]*CNT[u] for u in range(U)],[]))
        med=pts[n//2]
        if n%2==0: med=0.5*(pts[n//2-1]+med)
        s6=6.0*med
        for u in range(U):
            rj=RY[u]-FIT[u]
            if s6>0:
                t=abs(rj/s6); RW[u]=(1-t*t)*(1-t*t) if t<1.0 else 0.
            else: RW[u]=1. if rj==0 else 0.
    out=[]
    for d in range(D):
        xs=float(d); v=interp(RX,FIT,xs)
        if xs<=lb: v=FIT[0]
        if weighted and xs<X[inc]:
            v=interp(X,Y,xs)
            if xs<X[0]: v=Y[0]
        out.append(v)
    return np.array(out)

def random_column(rng):
    """A dispersion-vs-distance column like estimate_disp's: decaying,
    noisy, with NaN holes, sometimes rounded (ties, degenerate windows)."""
    D = int(rng.integers(5, 300))
    d = np.arange(D)
    col = 0.05 + 0.3 * np.exp(-d / rng.uniform(5, 80)) + \
        rng.normal(0, rng.uniform(0.001, 0.05), D)
    col = np.abs(col)
    col[rng.random(D) < rng.uniform(0, 0.3)] = np.nan
    if rng.random() < 0.2:
        col[:int(rng.integers(0, 5))] = np.nan
    if rng.random() < 0.1:
        col = np.round(col, 2)
    weighted = bool(rng.random() < 0.8)
    frac = -1. if rng.random() < 0.7 else float(rng.uniform(0.05, 0.8))
    return col, weighted, frac
