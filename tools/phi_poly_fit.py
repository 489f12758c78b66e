"""Near-minimax binary32 coefficients for the two series of qkd_spec.h's phi_core
(the certified interval iterations' phi): t(x) = (1 - e^-x) / x on [0, 0.35] and
h(s) = atanh(sqrt(s)) / sqrt(s) on [0, e^-2], relative error, leading coefficient
exactly 1. Lawson-reweighted least squares at Chebyshev nodes, coefficients rounded
to binary32 and locally searched (+-3 ulp) against the maximum error of binary32
Horner evaluation on 400k points. Prints the degree-4 fits (used) and degree-6
fits, and the error of the Taylor degree-6 forms they replaced. The bounds built on
them are certified on the GPU over every binary32 input
(tests/test_spec.py::test_phi_bounds_exhaustive), not by this script.
"""
import numpy as np
f32=np.float32
def horner32(c, x):
    p=np.full_like(x, c[-1])
    for cc in c[-2::-1]:
        p=(p.astype(np.float64)*x.astype(np.float64)+np.float64(cc)).astype(f32)
    return p
def fit(f, a, b, deg, n=6000):
    k=np.arange(n); x=(a+b)/2+(b-a)/2*np.cos(np.pi*(k+0.5)/n)
    y=f(x); V=np.vander(x,deg+1,increasing=True)
    # c0 fixed at 1
    w=np.ones(n)
    for it in range(300):
        W=np.sqrt(w)/np.abs(y)
        A=(V[:,1:]*W[:,None]); r=(y-1)*W
        c1,*_=np.linalg.lstsq(A, r, rcond=None)
        c=np.concatenate([[1.0],c1])
        e=np.abs(V@c-y)/np.abs(y)
        w=w*e; w/=w.sum()
    return c
def maxerr(c32, f, a, b):
    xs=np.linspace(a,b,400001).astype(f32)
    ys=f(xs.astype(np.float64))
    return np.max(np.abs(horner32(c32,xs).astype(np.float64)-ys)/ys)
def search(c, f, a, b, rounds=3):
    c32=c.astype(f32); best=maxerr(c32,f,a,b)
    for r in range(rounds):
        for i in range(1,len(c32)):
            for d in (-3,-2,-1,1,2,3):
                t=c32.copy(); t[i]=np.nextafter(t[i], np.inf if d>0 else -np.inf)
                for _ in range(abs(d)-1): t[i]=np.nextafter(t[i], np.inf if d>0 else -np.inf)
                e=maxerr(t,f,a,b)
                if e<best: best=e; c32=t
    return c32,best
t=lambda x: np.where(x==0,1.0,-np.expm1(-x)/np.where(x==0,1,x))
h=lambda s: np.where(s==0,1.0,np.arctanh(np.sqrt(s))/np.sqrt(np.where(s==0,1,s)))
for name,f,a,b,deg in [('t',t,0,0.35,4),('h',h,0,0.1354,4),('t',t,0,0.35,6),('h',h,0,0.1354,6)]:
    c=fit(f,a,b,deg); c32,e=search(c,f,a,b)
    print(name,deg,'%.3e'%e,[float(v).hex() for v in c32])
# current Taylor forms
tc=np.array([1,-0.5,1/6,-1/24,1/120,-1/720,1/5040],f32); hc=np.array([1,1/3,0.2,1/7,1/9,1/11,1/13],f32)
print('taylor t', '%.3e'%maxerr(tc,t,0,0.35), 'taylor h','%.3e'%maxerr(hc,h,0,0.1354))
