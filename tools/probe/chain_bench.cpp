// Microbenchmark: the XXH3 long-input scramble chain (8 accumulators, one
// step per 1 KiB block) on the host -- AVX-512DQ vpmullq, AVX-512F
// vpmuludq pair, scalar.  Build: g++ -O2 -o tools/probe/bin/chain_bench tools/probe/chain_bench.cpp
#include <immintrin.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <vector>
static const uint64_t SEC[8]={1,2,3,4,5,6,7,8};
constexpr uint64_t P=0x9E3779B1u;
__attribute__((target("avx512f,avx512dq"))) void chain512(const uint64_t*C, uint64_t nb, uint64_t*acc){
  __m512i a=_mm512_loadu_si512(acc); const __m512i s=_mm512_loadu_si512(SEC); const __m512i p=_mm512_set1_epi64(P);
  for(uint64_t b=0;b<nb;++b){ __m512i u=_mm512_add_epi64(a,_mm512_loadu_si512(C+8*b));
    __m512i x=_mm512_ternarylogic_epi64(u,_mm512_srli_epi64(u,47),s,0x96); a=_mm512_mullo_epi64(x,p);}
  _mm512_storeu_si512(acc,a);}
__attribute__((target("avx512f"))) void chain512b(const uint64_t*C, uint64_t nb, uint64_t*acc){
  __m512i a=_mm512_loadu_si512(acc); const __m512i s=_mm512_loadu_si512(SEC); const __m512i p=_mm512_set1_epi64(P);
  for(uint64_t b=0;b<nb;++b){ __m512i u=_mm512_add_epi64(a,_mm512_loadu_si512(C+8*b));
    __m512i x=_mm512_ternarylogic_epi64(u,_mm512_srli_epi64(u,47),s,0x96);
    __m512i lo=_mm512_mul_epu32(x,p); __m512i hi=_mm512_mul_epu32(_mm512_srli_epi64(x,32),p);
    a=_mm512_add_epi64(lo,_mm512_slli_epi64(hi,32));}
  _mm512_storeu_si512(acc,a);}
void chainsc(const uint64_t*C, uint64_t nb, uint64_t*acc){
  uint64_t a[8]; for(int j=0;j<8;++j)a[j]=acc[j];
  for(uint64_t b=0;b<nb;++b){ for(int j=0;j<8;++j){uint64_t u=a[j]+C[8*b+j]; a[j]=(u^(u>>47)^SEC[j])*P;}}
  for(int j=0;j<8;++j)acc[j]=a[j];}
int main(){ uint64_t nb=16<<20; std::vector<uint64_t> C(nb*8); for(size_t i=0;i<C.size();++i)C[i]=i*0x9E3779B97F4A7C15ull;
  for(int k=0;k<3;++k){ uint64_t a1[8]={0},a2[8]={0},a3[8]={0};
  auto t0=std::chrono::steady_clock::now(); chain512(C.data(),nb,a1); auto t1=std::chrono::steady_clock::now(); chain512b(C.data(),nb,a2); auto t2=std::chrono::steady_clock::now(); chainsc(C.data(),nb,a3); auto t3=std::chrono::steady_clock::now();
  printf("dq %.2f ns/blk  f %.2f  scalar %.2f  eq %d %d\n", std::chrono::duration<double,std::nano>(t1-t0).count()/nb, std::chrono::duration<double,std::nano>(t2-t1).count()/nb, std::chrono::duration<double,std::nano>(t3-t2).count()/nb, a1[3]==a3[3], a2[5]==a3[5]);}
}
