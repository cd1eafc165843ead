// merge_block.cc — see merge_block.h.
#include "merge_block.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace wtfgpu_host {

namespace {
constexpr uint64_t kDone = 1ull << 63;
}

MergeBlocks::MergeBlocks(uint64_t Cap) : cap_(Cap) {
  if (const char *e = getenv("WTF_MERGE_CAP")) {
    const uint64_t c = strtoull(e, nullptr, 0);
    if (c) cap_ = std::min(c, Cap);
  }
  if (cap_ == 0) cap_ = 1;
}

uint64_t MergeBlocks::Pack(const std::vector<uint64_t> &Extras, bool Done, uint64_t *Block) {
  if (head_ && head_ == carry_.size()) {  // drained: start over (no unbounded growth)
    carry_.clear();
    head_ = 0;
  }
  carry_.insert(carry_.end(), Extras.begin(), Extras.end());
  const uint64_t k = std::min<uint64_t>(Queued(), cap_);
  Block[0] = k | ((Done && Queued() == k) ? kDone : 0);
  if (k) memcpy(Block + 1, carry_.data() + head_, k * 8);
  head_ += k;
  if (head_ > (1u << 20) && head_ * 2 > carry_.size()) {  // compact the sent prefix now and then
    carry_.erase(carry_.begin(), carry_.begin() + (std::ptrdiff_t)head_);
    head_ = 0;
  }
  return 1 + k;
}

bool MergeBlocks::Unpack(const uint64_t *Blocks, size_t Words, uint64_t World, uint64_t Stride, uint64_t Cap,
                         std::vector<uint64_t> &All, bool *AllDone) {
  All.clear();
  bool all = true;
  size_t at = 0;
  for (uint64_t r = 0; r < World; r++) {
    if (Stride) at = (size_t)(r * Stride);
    if (at >= Words) return false;
    const uint64_t h = Blocks[at], k = h & ~kDone;
    if (k > Cap || at + 1 + k > Words || (Stride && 1 + k > Stride)) return false;
    all = all && (h & kDone);
    All.insert(All.end(), Blocks + at + 1, Blocks + at + 1 + k);
    at += 1 + k;
  }
  *AllDone = all;
  return true;
}

}  // namespace wtfgpu_host
