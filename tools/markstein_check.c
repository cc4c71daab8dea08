#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
// q = RN(c / den) via r = RN(1/den), q0 = RN(c*r), e = fma(-q0, den, c), q1 = fma(e, r, q0)
static inline uint64_t bits(double x){uint64_t u;memcpy(&u,&x,8);return u;}
static uint64_t s=88172645463325252ull; static inline uint64_t xr(){s^=s<<13;s^=s>>7;s^=s<<17;return s;}
int main(){
  long bad=0, badf=0, n=0;
  // every float w in [2^-10, 2^10) with stride, all c in 1..65
  for (uint32_t u = 0x3a800000u; u < 0x44800000u; u += 7) {
    float w; memcpy(&w,&u,4);
    double den = (double)w + 1e-9;
    double r = 1.0/den;
    for (int c=1;c<=65;++c){
      double q = (double)c/den;
      double q0 = (double)c*r;
      double e = fma(-q0, den, (double)c);
      double q1 = fma(e, r, q0);
      n++;
      if (bits(q)!=bits(q1)) { bad++; if ((float)q != (float)q1) badf++; }
    }
  }
  printf("n=%ld bad_double=%ld bad_float=%ld\n", n, bad, badf);
  // random doubles den in wide range incl. negative
  bad=0; badf=0; n=0;
  for (long i=0;i<200000000;i++){
    uint32_t u = (uint32_t)xr(); float w; memcpy(&w,&u,4);
    if (!isfinite(w)) continue;
    double den=(double)w+1e-9; if (den==0||!isfinite(1.0/den)) continue;
    double r=1.0/den; int c=1+(int)(xr()%65);
    double q=(double)c/den, q0=(double)c*r, e=fma(-q0,den,(double)c), q1=fma(e,r,q0);
    if (!isfinite(q)) continue;
    n++; if (bits(q)!=bits(q1)) {bad++; if ((float)q != (float)q1) badf++; if (bad<5) printf("w=%a c=%d q=%a q1=%a\n", w,c,q,q1);}
  }
  printf("random n=%ld bad_double=%ld bad_float=%ld\n", n, bad, badf);
}
