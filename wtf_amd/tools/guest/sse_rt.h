/* sse_rt.h — the guests' memcpy / memset, shaped like the vectorised runtime
 * routines the real targets call (vcruntime memcpy / memset, nt!RtlCopyMemory):
 * 16-byte SSE2 blocks (movdqu), a broadcast fill value (movd + punpck +
 * pshufd), then a byte tail. Built at gcc's default x86-64 SSE2 baseline, so
 * the synthetic snapshots run SSE code the way a Windows target does. */
#include <emmintrin.h>

static inline void sse_copy(unsigned char *D, const unsigned char *S, unsigned long long N) {
  unsigned long long I = 0;
  for (; I + 16 <= N; I += 16) _mm_storeu_si128((__m128i *)(D + I), _mm_loadu_si128((const __m128i *)(S + I)));
  for (; I < N; I++) D[I] = S[I];
}

static inline void sse_fill(unsigned char *D, int C, unsigned long long N) {
  const __m128i V = _mm_set1_epi8((char)C);
  unsigned long long I = 0;
  for (; I + 16 <= N; I += 16) _mm_storeu_si128((__m128i *)(D + I), V);
  for (; I < N; I++) D[I] = (unsigned char)C;
}
