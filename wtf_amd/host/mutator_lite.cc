// mutator_lite.cc — LibfuzzerMutator_t (wtf_api.h), the default mutator of a
// wtf target (targets.h:25, mutator.cc:8-54): one libFuzzer MutationDispatcher
// mutation (src/libs/libfuzzer/FuzzerMutate.cpp) of a corpus pick.
//
// Restated for bit-exact streams: the reference build of this very class is
// the checker (oracle/_ref/ref_hostcheck, tests/test_host_parity.py), so every
// draw of the generator happens in the reference's order, including the draws
// of mutators that end up failing, and the two pieces of state that outlive a
// call are kept as the reference keeps them:
//  * the scratch buffer (max_len bytes; bytes past the pick survive), and
//  * MutateInPlaceHere, which CrossOver and the in-place InsertPartOf write
//    and which CrossOver's copy modes then hand back whole (max_len bytes).
// With no custom mutator and no dictionaries (wtf registers none), the
// dispatcher's table is the 12 default mutators (FuzzerMutate.cpp:149-167);
// the two dictionary mutators always fail without drawing.
#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>

#include "wtf_api.h"

namespace {

enum Which_t : size_t {
  kEraseBytes, kInsertByte, kInsertRepeatedBytes, kChangeByte, kChangeBit, kShuffleBytes,
  kChangeASCIIInteger, kChangeBinaryInteger, kCopyPart, kCrossOver, kManualDict, kPersAutoDict,
  kNumMutators
};

template <typename T>
T bswap(T v) {
  if constexpr (sizeof(T) == 1) return v;
  else if constexpr (sizeof(T) == 2) return __builtin_bswap16(v);
  else if constexpr (sizeof(T) == 4) return __builtin_bswap32(v);
  else return __builtin_bswap64(v);
}

}  // namespace

// FuzzerMutate.cpp:182-186: a random byte, or one of the URL/format specials
uint8_t LibfuzzerMutator_t::RandCh() {
  if (RB()) return uint8_t(R(256));
  static const char Special[] = "!*'();:@&=+$,/?%#[]012Az-`~.\xff\x00";
  return uint8_t(Special[R(sizeof(Special) - 1)]);
}

// FuzzerMutate.cpp:422-433: overwrite a slice of To with a slice of From
size_t LibfuzzerMutator_t::CopyPartOf(const uint8_t *From, size_t FromSize, uint8_t *To, size_t ToSize) {
  const size_t ToBeg = R(ToSize);
  const size_t N = std::min(R(ToSize - ToBeg) + 1, FromSize);
  const size_t FromBeg = R(FromSize - N + 1);
  memmove(To + ToBeg, From + FromBeg, N);
  return ToSize;
}

// FuzzerMutate.cpp:437-460: insert a slice of From into To (0 when To is full)
size_t LibfuzzerMutator_t::InsertPartOf(const uint8_t *From, size_t FromSize, uint8_t *To, size_t ToSize,
                                        size_t MaxToSize) {
  if (ToSize >= MaxToSize) return 0;
  const size_t N = R(std::min(MaxToSize - ToSize, FromSize)) + 1;
  const size_t FromBeg = R(FromSize - N + 1);
  const size_t At = R(ToSize + 1);
  if (To == From) {  // the slice is parked in MutateInPlaceHere first
    InPlace_.resize(MaxToSize);
    memcpy(InPlace_.data(), From + FromBeg, N);
    memmove(To + At + N, To + At, ToSize - At);
    memmove(To + At, InPlace_.data(), N);
  } else {
    memmove(To + At + N, To + At, ToSize - At);
    memmove(To + At, From + FromBeg, N);
  }
  return ToSize + N;
}

// FuzzerMutate.cpp:18-48: alternate runs of A and B into Out
size_t LibfuzzerMutator_t::CrossOver(const uint8_t *A, size_t SizeA, const uint8_t *B, size_t SizeB, uint8_t *Out,
                                     size_t MaxOut) {
  MaxOut = R(MaxOut) + 1;
  size_t Pos[2] = {0, 0}, OutPos = 0;
  const uint8_t *Src[2] = {A, B};
  const size_t Len[2] = {SizeA, SizeB};
  for (int Side = 0; OutPos < MaxOut && (Pos[0] < SizeA || Pos[1] < SizeB); Side ^= 1) {
    if (Pos[Side] < Len[Side]) {
      const size_t N = R(std::min(MaxOut - OutPos, Len[Side] - Pos[Side])) + 1;
      memcpy(Out + OutPos, Src[Side] + Pos[Side], N);
      OutPos += N;
      Pos[Side] += N;
    }
  }
  return OutPos;
}

// FuzzerMutate.cpp:507-531
template <typename T>
size_t LibfuzzerMutator_t::ChangeBinaryInteger(uint8_t *Data, size_t Size) {
  if (Size < sizeof(T)) return 0;
  const size_t Off = R(Size - sizeof(T) + 1);
  T V;
  if (Off < 64 && !R(4)) {  // the testcase size, maybe byte-swapped
    V = T(Size);
    if (RB()) V = bswap(V);
  } else {  // add -10..10 in either byte order, maybe negate (always when +0)
    memcpy(&V, Data + Off, sizeof(T));
    T Add = T(R(21));
    Add -= 10;
    if (RB()) V = bswap(T(bswap(V) + Add));
    else V = T(V + Add);
    if (Add == 0 || RB()) V = T(~V);
  }
  memcpy(Data + Off, &V, sizeof(T));
  return Size;
}

// One mutator of the dispatcher table on Data[0, Size) with MaxSize_ bytes of
// room. 0 = it did not apply (FuzzerMutate.cpp:212-575).
size_t LibfuzzerMutator_t::Apply(size_t Which, uint8_t *Data, size_t Size) {
  const size_t Max = MaxSize_;
  switch (Which) {
    case kEraseBytes: {
      if (Size <= 1) return 0;
      const size_t N = R(Size / 2) + 1, At = R(Size - N + 1);
      memmove(Data + At, Data + At + N, Size - At - N);
      return Size - N;
    }
    case kInsertByte: {
      if (Size >= Max) return 0;
      const size_t At = R(Size + 1);
      memmove(Data + At + 1, Data + At, Size - At);
      Data[At] = RandCh();
      return Size + 1;
    }
    case kInsertRepeatedBytes: {
      if (Size + 3 >= Max) return 0;
      const size_t N = R(std::min<size_t>(Max - Size, 128) - 3 + 1) + 3;
      const size_t At = R(Size + 1);
      memmove(Data + At + N, Data + At, Size - At);
      const uint8_t B = RB() ? uint8_t(R(256)) : (RB() ? 0 : 255);  // 0x00 / 0xff favoured
      memset(Data + At, B, N);
      return Size + N;
    }
    case kChangeByte: {  // an empty testcase still gets Data[0] written (and fails)
      if (Size > Max) return 0;
      const size_t At = R(Size);
      Data[At] = RandCh();
      return Size;
    }
    case kChangeBit: {
      if (Size > Max) return 0;
      const size_t At = R(Size);
      Data[At] ^= uint8_t(1u << R(8));
      return Size;
    }
    case kShuffleBytes: {
      if (Size > Max || Size == 0) return 0;
      const size_t N = R(std::min<size_t>(Size, 8)) + 1;
      const size_t At = R(Size - N);
      std::shuffle(Data + At, Data + At + N, Rand_);
      return Size;
    }
    case kChangeASCIIInteger: {
      if (Size > Max) return 0;
      size_t B = R(Size);
      while (B < Size && !isdigit(Data[B])) B++;
      if (B == Size) return 0;
      size_t E = B;
      uint64_t V = 0;
      while (E < Size && isdigit(Data[E])) V = V * 10 + (Data[E++] - '0');
      switch (R(5)) {
        case 0: V++; break;
        case 1: V--; break;
        case 2: V /= 2; break;
        case 3: V *= 2; break;
        default: V = R(V * V); break;
      }
      for (size_t i = E; i-- > B;) {  // same width, rightmost digit first
        Data[i] = uint8_t('0' + V % 10);
        V /= 10;
      }
      return Size;
    }
    case kChangeBinaryInteger: {
      if (Size > Max) return 0;
      switch (R(4)) {
        case 3: return ChangeBinaryInteger<uint64_t>(Data, Size);
        case 2: return ChangeBinaryInteger<uint32_t>(Data, Size);
        case 1: return ChangeBinaryInteger<uint16_t>(Data, Size);
        default: return ChangeBinaryInteger<uint8_t>(Data, Size);
      }
    }
    case kCopyPart: {
      if (Size > Max || Size == 0) return 0;
      if (Size == Max || RB()) return CopyPartOf(Data, Size, Data, Size);
      return InsertPartOf(Data, Size, Data, Size, Max);
    }
    case kCrossOver: {
      if (Size > Max || Size == 0 || !HasCrossOver_ || CrossOverWith_.empty()) return 0;
      const uint8_t *O = CrossOverWith_.data();
      const size_t OSize = CrossOverWith_.size();
      InPlace_.resize(Max);
      uint8_t *U = InPlace_.data();
      size_t N = 0;
      switch (R(3)) {
        case 0: N = CrossOver(Data, Size, O, OSize, U, Max); break;
        case 1:  // U is max_len long: the insert never fits, the copy runs
          N = InsertPartOf(O, OSize, U, Max, Max);
          if (!N) N = CopyPartOf(O, OSize, U, Max);
          break;
        default: N = CopyPartOf(O, OSize, U, Max); break;
      }
      memcpy(Data, U, N);
      return N;
    }
    default:  // kManualDict, kPersAutoDict: empty dictionaries
      return 0;
  }
}

// mutator.cc:21-44 + FuzzerMutate.cpp:633-652 (MutateImpl)
std::string LibfuzzerMutator_t::GetNewTestcase(const Corpus_t &Corpus) {
  const Testcase_t *T = Corpus.PickTestcase();
  if (!T) {
    printf("The corpus is empty, exiting\n");
    std::abort();
  }
  // the reference memcpy's the pick into a max_len buffer; a longer pick is
  // clipped here instead of overflowing it
  const size_t In = std::min(T->BufferSize_, MaxSize_);
  if (In) memcpy(Scratch_.data(), T->Buffer_.get(), In);
  uint8_t *Data = Scratch_.data();
  for (int Try = 0; Try < 100; Try++) {
    const size_t N = Apply(R(kNumMutators), Data, In);
    if (N && N <= MaxSize_) return std::string((const char *)Data, N);
  }
  Data[0] = ' ';  // every attempt failed (FuzzerMutate.cpp:650-651)
  return std::string((const char *)Data, 1);
}
