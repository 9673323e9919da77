"""RadTan unproject on config 4's own pixels, replayed on the CPU (numpy):
the reference's Newton loop (rad_tan.rs:436-518) step histogram and the
certified fast loop's (camera_models.hpp RadTan::newton_fast) fallback rate,
decisions replicated in numpy float64 (the rounding of the fast loop's FMAs
is not replicated: its decisions are certified against a band far wider
than that).  1M synthetic points (the bench distribution), projected by
the oracle; only Ok projections are unprojected.

  python tools/diag_radtan_steps.py
"""
import numpy as np, sys
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
import oracle as O
from apex_camera_models import samples
params,(w,h)=samples.SAMPLES[1]
n=1_000_000
pts=samples.synthetic_points(n, offset=0)
uv,st,_=O.project(1,params,w,h,pts)
ok=st==0
print("project ok", ok.mean())
uvk=uv[ok]
fx,fy,cx,cy,k1,k2,p1,p2,k3=params
tx=(uvk[:,0]-cx)/fx; ty=(uvk[:,1]-cy)/fy
x=tx.copy(); y=ty.copy()
N=len(x)
done=np.zeros(N,bool); steps=np.zeros(N,int); status=np.zeros(N,int)
for it in range(100):
    a=~done
    xx=x[a]; yy=y[a]
    r2=xx*xx+yy*yy; r4=r2*r2; r6=r4*r2
    rad=1+k1*r2+k2*r4+k3*r6
    xe=xx*rad+2*p1*xx*yy+p2*(r2+2*xx*xx); ye=yy*rad+p1*(r2+2*yy*yy)+2*p2*xx*yy
    ex=xe-tx[a]; ey=ye-ty[a]
    conv=np.sqrt(ex*ex+ey*ey)<1e-6
    idx=np.nonzero(a)[0]
    done[idx[conv]]=True; steps[idx[conv]]=it
    b=~conv; idx=idx[b]; xx=xx[b]; yy=yy[b]; r2=r2[b]; r4=r4[b]; rad=rad[b]; ex=ex[b]; ey=ey[b]
    ddx=(k1+2*k2*r2+3*k3*r4)*2*xx; ddy=(k1+2*k2*r2+3*k3*r4)*2*yy
    j00=rad+xx*ddx+2*p1*yy+p2*(2*xx+4*xx); j01=xx*ddy+2*p1*xx+p2*2*yy
    j10=yy*ddx+p1*2*xx+2*p2*yy; j11=rad+yy*ddy+p1*(2*yy+4*yy)+2*p2*xx
    det=j00*j11-j10*j01
    dx=(j11*ex-j01*ey)/det; dy=(-j10*ex+j00*ey)/det
    x[idx]-=dx; y[idx]-=dy
    c2=np.sqrt(dx*dx+dy*dy)<1e-6
    done[idx[c2]]=True; steps[idx[c2]]=it+1
status[~done]=4
print("pixels",N,"fail(100 its)",(~done).mean())
h=np.bincount(steps[done]); print("steps hist", h[:20])
# waves of 64 (pixels in order of the synthetic cloud) containing >=1 failure
f=~done
W=N//64; fw=f[:W*64].reshape(W,64).any(1).mean(); print("waves with a failing pixel", fw)
mx=np.where(done, steps, 100)[:W*64].reshape(W,64).max(1); print("mean wave max steps", mx.mean(), "mean steps", np.where(done,steps,100).mean())
r=np.sqrt(tx**2+ty**2); print("fail r range", r[f].min() if f.any() else None, r[f].max() if f.any() else None)
# replica of RadTan::newton_fast certification (fma ~ plain ops here; decisions only)
tol2=float.fromhex('0x1.19799812dea10p-40'); lo=tol2*(1-2**-10); hi=tol2*(1+2**-10)
x=tx.copy(); y=ty.copy(); state=np.zeros(N,int); nst=np.zeros(N,int)
k2d=2*k2; k3t=3*k3; p1d=2*p1; p2d=2*p2; p1s=6*p1; p2s=6*p2
for i in range(12):
    a=state==0
    xx=x[a]; yy=y[a]; idx=np.nonzero(a)[0]
    x2=xx*xx; y2=yy*yy; xy=xx*yy; s=x2+y2
    rad=((k3*s+k2)*s+k1)*s+1
    xe=xx*rad+(p1d*xy+p2*((xx+xx)*xx+s)); ye=yy*rad+(p1*((yy+yy)*yy+s)+p2d*xy)
    ex=xe-tx[a]; ey=ye-ty[a]; en2=ex*ex+ey*ey
    st=np.full(len(idx),0)
    bad=~((np.abs(xx)<=2)&(np.abs(yy)<=2))
    st[bad]=2
    c1=(~bad)&(en2<lo); st[c1]=1
    band=(~bad)&(~c1)&~(en2>hi); st[band]=2
    go=(~bad)&(~c1)&(~band)
    cm=(k3t*s+k2d)*s+k1; w_=cm+cm
    j00=(x2*w_+rad)+(p1d*yy+p2s*xx); j11=(y2*w_+rad)+(p1s*yy+p2d*xx); j01=xy*w_+(p1d*xx+p2d*yy)
    det=j00*j11-j01*j01; sj=np.abs(j00)+np.abs(j11)+2*np.abs(j01)
    okd=(np.abs(det)>=0.0625)&(sj<=64)
    st[go&~okd]=2
    g2=go&okd
    dx=(j11*ex-j01*ey)/det; dy=(j00*ey-j01*ex)/det
    xn=xx-dx; yn=yy-dy; dn2=dx*dx+dy*dy
    st[g2]=np.where(dn2[g2]<lo,1,np.where(dn2[g2]>hi,0,2))
    x[idx[g2]]=xn[g2]; y[idx[g2]]=yn[g2]
    state[idx]=st; nst[idx]+=1
fallback=state!=1
print("fast-loop fallback fraction", fallback.mean(), " of which nan", np.isnan(tx[fallback]).mean() if fallback.any() else 0)
print("waves with a fallback pixel", fallback[:W*64].reshape(W,64).any(1).mean())
print("fast steps hist", np.bincount(nst[~fallback])[:15], "wave-max mean", nst[:W*64].reshape(W,64).max(1).mean())
