/* sse_rt.h — the guests' memcpy / memset, shaped like the vectorised runtime
 * routines the real targets call (vcruntime memcpy / memset, nt!RtlCopyMemory
 * on an AVX2 machine): 32-byte AVX2 blocks (vmovdqu ymm), 16-byte SSE2 blocks
 * (movdqu), a broadcast fill value (vpbroadcastb / punpck + pshufd), a byte
 * tail, and vzeroupper before returning to SSE code. The rest of the guest is
 * built at gcc's default x86-64 SSE2 baseline. */
#include <immintrin.h>

__attribute__((target("avx2"))) static inline void sse_copy(unsigned char *D, const unsigned char *S,
                                                            unsigned long long N) {
  unsigned long long I = 0;
  if (N >= 32) {
    for (; I + 32 <= N; I += 32)
      _mm256_storeu_si256((__m256i *)(D + I), _mm256_loadu_si256((const __m256i *)(S + I)));
    _mm256_zeroupper();
  }
  for (; I + 16 <= N; I += 16) _mm_storeu_si128((__m128i *)(D + I), _mm_loadu_si128((const __m128i *)(S + I)));
  for (; I < N; I++) D[I] = S[I];
}

__attribute__((target("avx2"))) static inline void sse_fill(unsigned char *D, int C, unsigned long long N) {
  unsigned long long I = 0;
  if (N >= 32) {
    const __m256i V = _mm256_set1_epi8((char)C);
    for (; I + 32 <= N; I += 32) _mm256_storeu_si256((__m256i *)(D + I), V);
    _mm256_zeroupper();
  }
  const __m128i V = _mm_set1_epi8((char)C);
  for (; I + 16 <= N; I += 16) _mm_storeu_si128((__m128i *)(D + I), V);
  for (; I < N; I++) D[I] = (unsigned char)C;
}
