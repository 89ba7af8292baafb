// Exhaustive-ish check that the FMA (Markstein) division used by k_integrate
// (kfx_kernels.hip div_rn) equals IEEE division for its divisors.
// gcc -O2 -ffp-contract=off -mfma tools/markstein_check.c -lm && ./a.out
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <stdlib.h>
static float bits(uint32_t u){float f; memcpy(&f,&u,4); return f;}
static uint64_t s=88172645463325252ULL; static uint32_t rnd(){ s^=s<<13; s^=s>>7; s^=s<<17; return (uint32_t)s; }
int main(){
  long bad=0, tot=0;
  float divs[70]; int nd=0;
  for(int d=1; d<=65; ++d) divs[nd++]=(float)d;
  divs[nd++]=2.1f*3.0f/512.0f; divs[nd++]=2.1f*2.048f/512.0f; divs[nd++]=2.1f*2.048f/1024.0f; divs[nd++]=2.1f*4.096f/2048.0f;
  for(int k=0;k<nd;++k){
    float d=divs[k]; float y=1.0f/d;
    // exhaustive over all positive floats in [2^-20, 2^20) with stride, plus random
    for(uint32_t u=0x35800000u; u<0x49800000u; u+=7){  // ~2^-20 .. 2^20
      for(int sg=0; sg<2; ++sg){
        float x = sg? -bits(u): bits(u);
        float q0=x*y; float r=fmaf(-q0,d,x); float q1=fmaf(r,y,q0);
        float e=x/d; tot++;
        if(memcmp(&q1,&e,4)) { if(bad<5) printf("mismatch d=%g x=%a q1=%a exact=%a\n",d,x,q1,e); bad++; }
      }
    }
    for(int i=0;i<2000000;++i){ float x=bits(rnd()); if(!isfinite(x)||fabsf(x)>1e30f||fabsf(x)<1e-30f) continue; float q0=x*y; float r=fmaf(-q0,d,x); float q1=fmaf(r,y,q0); float e=x/d; tot++; if(memcmp(&q1,&e,4)){ if(bad<5) printf("mismatch rnd d=%g x=%a\n",d,x); bad++;} }
  }
  printf("tested %ld, mismatches %ld\n", tot, bad);
  // colour: trunc(m/c) for all m in [0, 255*64+255], c in [2,65] via Markstein
  long cb=0; for(int c=2;c<=65;++c){ float y=1.0f/(float)c; for(int m=0;m<=255*65+255;++m){ float x=(float)m; float q0=x*y; float r=fmaf(-q0,(float)c,x); float q1=fmaf(r,y,q0); if((uint8_t)q1 != (uint8_t)(x/(float)c)) cb++; } }
  printf("colour mismatches %ld\n", cb);
  return 0;
}
