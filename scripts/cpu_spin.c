#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
static void* run(void* a){ volatile unsigned long x=0; for(unsigned long i=0;i<400000000UL;++i) x+=i; return 0;}
int main(int c,char**v){int T=atoi(v[1]); pthread_t t[64]; struct timespec a,b; clock_gettime(CLOCK_MONOTONIC,&a);
for(int i=0;i<T;i++) pthread_create(&t[i],0,run,0); for(int i=0;i<T;i++) pthread_join(t[i],0);
clock_gettime(CLOCK_MONOTONIC,&b); printf("T=%d %.3f s\n",T,(b.tv_sec-a.tv_sec)+(b.tv_nsec-a.tv_nsec)*1e-9);}
