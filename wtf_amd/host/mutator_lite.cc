// mutator_lite.cc — LibfuzzerMutator_t (wtf_api.h): the default mutator of a
// target, restating the mutation kinds of libFuzzer's MutationDispatcher
// (FuzzerMutate.cpp, vendored by the reference as its default through
// mutator.cc:8-51) in a reduced form.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "wtf_api.h"

size_t LibfuzzerMutator_t::MutateOnce(std::vector<uint8_t> &D, size_t Size) {
  // D has MaxSize_ bytes of room; returns the new size or 0 if this kind did not apply
  switch (R(9)) {
    case 0: {  // EraseBytes
      if (Size <= 1) return 0;
      const size_t N = 1 + R(Size / 2), Idx = R(Size - N + 1);
      std::copy(D.begin() + Idx + N, D.begin() + Size, D.begin() + Idx);
      return Size - N;
    }
    case 1: {  // InsertByte
      if (Size >= MaxSize_) return 0;
      const size_t Idx = R(Size + 1);
      std::copy_backward(D.begin() + Idx, D.begin() + Size, D.begin() + Size + 1);
      D[Idx] = (uint8_t)R(256);
      return Size + 1;
    }
    case 2: {  // InsertRepeatedBytes
      if (Size + 3 > MaxSize_) return 0;
      const size_t N = std::min<size_t>(3 + R(126), MaxSize_ - Size), Idx = R(Size + 1);
      std::copy_backward(D.begin() + Idx, D.begin() + Size, D.begin() + Size + N);
      const uint8_t B = R(2) ? (uint8_t)R(256) : (R(2) ? 0 : 0xff);
      std::fill(D.begin() + Idx, D.begin() + Idx + N, B);
      return Size + N;
    }
    case 3:  // ChangeByte
      if (!Size) return 0;
      D[R(Size)] = (uint8_t)R(256);
      return Size;
    case 4:  // ChangeBit
      if (!Size) return 0;
      D[R(Size)] ^= (uint8_t)(1u << R(8));
      return Size;
    case 5: {  // ShuffleBytes
      if (!Size) return 0;
      const size_t N = 1 + R(std::min<size_t>(Size, 8)), Idx = R(Size - N + 1);
      std::shuffle(D.begin() + Idx, D.begin() + Idx + N, Rand_);
      return Size;
    }
    case 6: {  // ChangeBinaryInteger: add a small delta to a 1/2/4/8-byte integer
      const size_t W = (size_t)1 << R(4);
      if (Size < W) return 0;
      const size_t Idx = R(Size - W + 1);
      uint64_t V = 0;
      memcpy(&V, &D[Idx], W);
      if (R(4) == 0) V = (uint64_t)Size;
      else V += (uint64_t)((int64_t)R(21) - 10);
      memcpy(&D[Idx], &V, W);
      return Size;
    }
    case 7: {  // CopyPart (overwrite)
      if (Size < 2) return 0;
      const size_t N = 1 + R(Size - 1), From = R(Size - N + 1), To = R(Size - N + 1);
      std::vector<uint8_t> T(D.begin() + From, D.begin() + From + N);
      std::copy(T.begin(), T.end(), D.begin() + To);
      return Size;
    }
    default: {  // CrossOver with the last testcase that found new coverage
      if (CrossOverWith_.empty()) return 0;
      const size_t N = std::min(CrossOverWith_.size(), MaxSize_);
      const size_t Cut = R(std::min(Size, N) + 1);
      std::copy(CrossOverWith_.begin() + Cut, CrossOverWith_.begin() + N, D.begin() + Cut);
      return N;
    }
  }
}

std::string LibfuzzerMutator_t::GetNewTestcase(const Corpus_t &Corpus) {
  const Testcase_t *T = Corpus.PickTestcase();
  if (!T) {
    printf("The corpus is empty, exiting\n");
    std::abort();
  }
  std::vector<uint8_t> D(std::max<size_t>(MaxSize_, T->BufferSize_));
  std::copy(T->Buffer_.get(), T->Buffer_.get() + T->BufferSize_, D.begin());
  size_t Size = T->BufferSize_, New = 0;
  for (int Try = 0; Try < 100 && !New; Try++) New = MutateOnce(D, Size);
  if (New) Size = New;
  return std::string((const char *)D.data(), std::min(Size, MaxSize_));
}
