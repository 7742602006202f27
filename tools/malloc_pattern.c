/* malloc_pattern.c — what glibc charges for the socket layer's batch pattern:
 * 8192 blocks of ~0.2-1.2 KB allocated, then all freed (a burst's batches and
 * their reclaim).  Diagnostics for host/nstack.c bp_alloc.
 *   gcc -O2 tools/malloc_pattern.c -o /tmp/malloc_pattern */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
static double now(){struct timespec t;clock_gettime(CLOCK_MONOTONIC,&t);return t.tv_sec*1e9+t.tv_nsec;}
int main(){
  enum{N=8192,R=50}; void*p[N];
  for(int sz=200; sz<=1200; sz+=500){
  double tm=0,tf=0;
  for(int r=0;r<R;r++){
    double a=now();
    for(int i=0;i<N;i++){p[i]=malloc(sz+(i&3)*104); memset(p[i],0,64);}
    double b=now();
    for(int i=0;i<N;i++) free(p[(i*7919)%N]);
    double c=now(); if(r>2){tm+=b-a;tf+=c-b;}
  }
  printf("size~%d: malloc %.1f ns, free %.1f ns\n", sz, tm/(R-3)/N, tf/(R-3)/N);}
}
