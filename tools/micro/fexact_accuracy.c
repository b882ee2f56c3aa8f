// Development aid (host, gcc -O2 ... -lm): accuracy of the exact-f SCL boxplus forms of
// csrc/softplus.h (Taylor, economised P9/R10) against long double, and the reference expression.
// Generated from tools/cheb_coeffs.py output; DESIGN.md section 3.2 quotes its numbers.

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static const double R10[]={0.6666666666666666,0.39999999999999514,0.28571428571603413,0.22222222197853667,0.18181819920440906,0.15384543207664578,0.133351941539121,0.11734082174871642,0.10846687166200544,0.07485743922141379,0.1564211337480669}, P9[]={0.5000000000000001,0.1666666666666667,0.04166666666662413,0.008333333333326136,0.001388888891721154,0.00019841269874817515,2.4801521299750923e-05,2.75572554044176e-06,2.7620086491464514e-07,2.5105215165649368e-08}, P10[]={0.5,0.1666666666666667,0.04166666666666668,0.008333333333326136,0.0013888888888879075,0.00019841269874817515,2.480158733643862e-05,2.75572554044176e-06,2.755726328311978e-07,2.5105215165649368e-08,2.0918136198258855e-09};
static double horner(const double* c,int n,double x){double p=c[n-1];for(int i=n-2;i>=0;i--)p=fma(p,x,c[i]);return p;}
static double fnew(double x,double y,double lmax,const double*P,int np,const double*R,int nr){
 double xc=fmax(fmin(x,lmax),-lmax),yc=fmax(fmin(y,lmax),-lmax);double a=fabs(xc),b=fabs(yc);double m=fmin(a,b),M=fmax(a,b);
 const double L2E=1.4426950408889634,hi=0x1.62e42fefa39efp-1,lo=0x1.abc9e3b39803fp-56;
 double ze=m-M,zm=-2.0*m; double ke=rint(ze*L2E),km=rint(zm*L2E);
 double re=fma(-ke,hi,ze); re=fma(-ke,lo,re); double rm=fma(-km,hi,zm); rm=fma(-km,lo,rm);
 double pe=horner(P,np,re), pm=horner(P,np,rm);
 double E=ldexp(fma(re*re,pe,re)+1.0,(int)ke);
 double tk=ldexp(1.0,(int)km); double G=-fma(tk,fma(rm*rm,pm,rm),tk-1.0);
 double eg=E*G; double den=fma(2.0,E,2.0)-eg; double s=-eg/den; double w=s*s; double Rv=horner(R,nr,w);
 double v=m+fma(s*w,Rv,s+s); return ((xc<0)!=(yc<0))?-v:v;}
static long double fexact(double x,double y,double lmax){long double xc=fmaxl(fminl(x,lmax),-lmax),yc=fmaxl(fminl(y,lmax),-lmax);long double a=fabsl(xc),b=fabsl(yc),m=fminl(a,b),M=fmaxl(a,b);
long double v=m+log1pl(expl(-(M+m)))-log1pl(expl(-(M-m)));return ((xc<0)!=(yc<0))?-v:v;}
static double fref(double x,double y,double lmax){double xc=fmax(fmin(x,lmax),-lmax),yc=fmax(fmin(y,lmax),-lmax);return log(1.0+exp(xc+yc))-log(exp(xc)+exp(yc));}
int main(){
 /* taylor reference coefficient sets */
 double PT[12],RT[17]; {double f=2; for(int i=0;i<12;i++){PT[i]=1.0/f; f*=(i+3);} for(int i=0;i<17;i++) RT[i]=2.0/(2*i+3);}
 struct {const char*n;const double*P;int np;const double*R;int nr;} cfg[]={{"taylor",PT,12,RT,17},{"P9R10",P9,10,R10,11},{"P10R10",P10,11,R10,11}};
 for(int c=0;c<3;c++){srand(1);double mx=0,mxsmall=0;long double sum=0;int N=4000000;
  for(int i=0;i<N;i++){double sc=pow(10.0,(rand()/(double)RAND_MAX)*4-3);double x=((rand()/(double)RAND_MAX)*2-1)*sc*20,y=((rand()/(double)RAND_MAX)*2-1)*sc*20; if(i%7==0) y=x*(1+1e-9*(rand()/(double)RAND_MAX));
   long double e=fexact(x,y,30.0);double d=fabsl(fnew(x,y,30.0,cfg[c].P,cfg[c].np,cfg[c].R,cfg[c].nr)-e);if(d>mx)mx=d;sum+=d;
   /* error in ulps of max(|e|, 1e-3) small-magnitude region */
  }
  printf("%-8s max abs err %.3g mean %.3g\n",cfg[c].n,mx,(double)(sum/N));}
 srand(1);double mr=0;long double sr=0;int N=4000000;for(int i=0;i<N;i++){double sc=pow(10.0,(rand()/(double)RAND_MAX)*4-3);double x=((rand()/(double)RAND_MAX)*2-1)*sc*20,y=((rand()/(double)RAND_MAX)*2-1)*sc*20;if(i%7==0) y=x*(1+1e-9*(rand()/(double)RAND_MAX));long double e=fexact(x,y,30.0);double d=fabsl(fref(x,y,30.0)-e);if(d>mr)mr=d;sr+=d;}
 printf("ref-form max abs err %.3g mean %.3g\n",mr,(double)(sr/N));
 return 0;}
