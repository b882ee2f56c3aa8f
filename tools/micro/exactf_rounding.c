// Development aid (host, gcc -O2 ... -lm): correct rounding of csrc/exactf.h exp_cr / log_cr
// (economised) and the Taylor forms they replaced, against expl / logl rounded to fp32, 5e7
// arguments each.  The reciprocal is emulated by an fp32 one (coarser than v_rcp_f64).

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
static const double E10[]={1.0,1.0000000000000067,0.5000000000000019,0.16666666666554325,0.041666666666487974,0.008333333385695266,0.001388888895234707,0.00019841170236135905,2.480148544815057e-05,2.7640194893802356e-06,2.763265216957956e-07}, RL5[]={0.6666666666666206,0.40000000011263015,0.2857142412272895,0.22222863785496652,0.18140134518808063,0.16622633991749486};
static float exp_old(float xf){double x=xf;const double L2E=1.4426950408889634,hi=0x1.62e42fefa39efp-1,lo=0x1.abc9e3b39803fp-56;double k=rint(x*L2E);double r=fma(-k,hi,x);r=fma(-k,lo,r);
 double p=2.505210838544172e-08;double cc[]={2.755731922398589e-07,2.7557319223985893e-06,2.48015873015873e-05,0.0001984126984126984,0.001388888888888889,0.008333333333333333,0.041666666666666664,0.16666666666666666,0.5,1.0,1.0};for(int i=0;i<11;i++)p=fma(p,r,cc[i]);return ldexpf((float)p,(int)k);}
static float exp_new(float xf){double x=xf;const double L2E=1.4426950408889634,hi=0x1.62e42fefa39efp-1,lo=0x1.abc9e3b39803fp-56;double k=rint(x*L2E);double r=fma(-k,hi,x);r=fma(-k,lo,r);
 double p=E10[10];for(int i=9;i>=0;i--)p=fma(p,r,E10[i]);return ldexpf((float)p,(int)k);}
static float log_old(float xf){const double hi=0x1.62e42fefa39efp-1,lo=0x1.abc9e3b39803fp-56;int e;double m=frexp((double)xf,&e);if(m<0.70710678118654752){m=m+m;e-=1;}double f=m-1.0;double s=f/(2.0+f);double z=s*s;
 double R=2.0/19.0;double cc[]={2.0/17,2.0/15,2.0/13,2.0/11,2.0/9,2.0/7,2.0/5,2.0/3};for(int i=0;i<8;i++)R=fma(R,z,cc[i]);double lm=fma(s*z,R,s+s);double de=e;return (float)fma(de,hi,fma(de,lo,lm));}
static double rcp_approx(double d){float f=(float)(1.0/d);return (double)f;} /* stands in for v_rcp_f64 (worse than the hardware's) */
static float log_new(float xf){const double hi=0x1.62e42fefa39efp-1,lo=0x1.abc9e3b39803fp-56;int e;double m=frexp((double)xf,&e);if(m<0.70710678118654752){m=m+m;e-=1;}double f=m-1.0;double den=2.0+f;
 double rc=rcp_approx(den);double t=fma(-den,rc,1.0);rc=fma(rc,t,rc);t=fma(-den,rc,1.0);rc=fma(rc,t,rc);double q=f*rc;double s=fma(rc,fma(-den,q,f),q);double z=s*s;
 double R=RL5[5];for(int i=4;i>=0;i--)R=fma(R,z,RL5[i]);double lm=fma(s*z,R,s+s);double de=e;return (float)fma(de,hi,fma(de,lo,lm));}
static uint64_t st=88172645463325252ull; static uint32_t rnd(){st^=st<<13;st^=st>>7;st^=st<<17;return (uint32_t)(st>>11);}
int main(){long N=50000000;long be_o=0,be_n=0,bl_o=0,bl_n=0;
 for(long i=0;i<N;i++){ /* exp args: uniform in [-87,87] plus small */
  float x=((rnd()/4294967296.0)*2-1)*(i%3==0?87.0f:(i%3==1?4.0f:0.01f));
  float cr=(float)expl((long double)x); if(exp_old(x)!=cr)be_o++; if(exp_new(x)!=cr)be_n++;
  uint32_t b=rnd()&0x7fffffff; float y; memcpy(&y,&b,4); if(!(y>0)||isinf(y)||isnan(y)||y<1e-30f) y=1.0f+(rnd()/4294967296.0f);
  float lcr=(float)logl((long double)y); if(log_old(y)!=lcr)bl_o++; if(log_new(y)!=lcr)bl_n++;}
 printf("exp misrounded: old %ld new %ld of %ld; log misrounded: old %ld new %ld\n",be_o,be_n,N,bl_o,bl_n);return 0;}
