"""Development aid: Chebyshev economisation (exact rational arithmetic) of the power series behind
the exact-f polynomials of csrc/softplus.h: P(r) = (e^r - 1 - r)/r^2 on |r| <= ln2/2 and the atanh
series R(w) = sum 2/(2i+3) w^i on [0, 1/9]; prints the tail bound per degree and writes the
double coefficients to /tmp/cheb.json.  python tools/cheb_coeffs.py"""
from fractions import Fraction as F
import math
def poly_mul(a,b):
    r=[F(0)]*(len(a)+len(b)-1)
    for i,x in enumerate(a):
        for j,y in enumerate(b): r[i+j]+=x*y
    return r
def cheb_T(n):  # monomial coeffs of T_n(u)
    T=[[F(1)],[F(0),F(1)]]
    for k in range(2,n+1):
        a=poly_mul([F(0),F(2)],T[k-1]); b=T[k-2]+[F(0)]*(len(a)-len(T[k-2]))
        T.append([x-y for x,y in zip(a,b)])
    return T
def economize(coef, lo, hi, tol):
    # coef: monomial in x on [lo,hi]; substitute x = c + d*u, u in [-1,1]
    c=(F(lo)+F(hi))/2; d=(F(hi)-F(lo))/2
    N=len(coef)-1
    # p(u) = sum coef_i (c + d u)^i
    pu=[F(0)]*(N+1)
    binom=[[F(0)]*(N+1) for _ in range(N+1)]
    for i,a in enumerate(coef):
        # (c+du)^i
        for k in range(i+1):
            pu[k]+=a*math.comb(i,k)*c**(i-k)*d**k
    T=cheb_T(N)
    # convert pu monomial(u) -> chebyshev coefficients: solve from top
    ch=[F(0)]*(N+1); rem=pu[:]
    for k in range(N,-1,-1):
        lead=T[k][k]
        ch[k]=rem[k]/lead
        for j in range(k+1): rem[j]-=ch[k]*T[k][j]
    return ch,c,d,T
def back(ch,D,c,d,T):
    pu=[F(0)]*(D+1)
    for k in range(D+1):
        for j in range(k+1): pu[j]+=ch[k]*T[k][j]
    # u = (x - c)/d -> monomial in x
    px=[F(0)]*(D+1)
    for k,a in enumerate(pu):
        # ((x-c)/d)^k
        for j in range(k+1):
            px[j]+=a*math.comb(k,j)*(-c)**(k-j)/d**k
    return px
def report(name, coef, lo, hi, Ds):
    ch,c,d,T=economize(coef,lo,hi,0)
    for D in Ds:
        tail=sum(abs(x) for x in ch[D+1:])
        print(name, 'degree',D,'tail bound %.3g'%float(tail))
    return ch,c,d,T
# R(w) = sum 2/(2i+3) w^i, w in [0,1/9]
R=[F(2,2*i+3) for i in range(40)]
chR=report('R', R, 0, F(1,9), range(8,17))
# P(r) = sum r^i/(i+2)!, |r| <= ln2/2 (use 0.3466 rational bound slightly larger)
P=[F(1,math.factorial(i+2)) for i in range(30)]
chP=report('P', P, -F(3466,10000), F(3466,10000), range(7,13))
import pickle
pickle.dump((chR,chP),open('/tmp/cheb.pkl','wb'))
# pm_log R(z)= sum_{i>=1} 2/(2i+1) z^(i-1), z in [0, 0.17158^2]
zmax=F(17158,100000)**2
RL=[F(2,2*i+1) for i in range(1,40)]
chL=report('RL', RL, 0, zmax, range(4,12))
def coeffs(chtuple, D):
    ch,c,d,T=chtuple
    px=back(ch,D,c,d,T)
    return [float(x) for x in px]
import json
out={'R10':coeffs(chR,10),'P9':coeffs(chP,9),'P10':coeffs(chP,10),'RL6':coeffs(chL,6),'RL7':coeffs(chL,7)}
json.dump(out,open('/tmp/cheb.json','w'))
for k,v in out.items(): print(k,[repr(x) for x in v])

# exactf.h (exact-f SC: fp32 results of fp64 evaluations, error target < 2^-46 relative):
# e^r itself on |r| <= ln2/2, and the log series RL on [0, 0.17158^2]
E = [F(1, math.factorial(i)) for i in range(30)]
chE = report('E', E, -F(3466, 10000), F(3466, 10000), range(8, 12))
out2 = {'E10': coeffs(chE, 10), 'RL5': coeffs(chL, 5)}
json.dump(out2, open('/tmp/cheb2.json', 'w'))
for k, v in out2.items():
    print(k, [repr(x) for x in v])
