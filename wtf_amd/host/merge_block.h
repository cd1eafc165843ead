// merge_block.h — the per-rank block of one deferred coverage merge (SURVEY
// 8(e)): every step each shard sends one block, and every shard reads every
// shard's block back in rank order.
//
// A block is u64 words: a header (count | done << 63), then `count` coverage
// values from outside the map (the overflow list: rips on pages outside the
// slot table, --edges values). At most `Cap` values travel per block; the
// rest stay queued, in order, for the next merges. A shard says "done" only
// in a block that empties its queue, so no shard stops while values it owes
// the others are still queued (the reference master's aggregate gets every
// value, server.h:816-854).
//
// Host-only: the RCCL exchange (rccl_exchange.cc) all-gathers fixed-size
// blocks on the device, the TCP exchange of the CPU twins (runner.cc) sends
// them packed; both pack and read them here.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace wtfgpu_host {

constexpr uint64_t kMergeCap = 4096;  // overflow values per shard per merge (the rest wait their turn)

class MergeBlocks {
 public:
  // WTF_MERGE_CAP in the environment overrides Cap (tests drain small caps)
  explicit MergeBlocks(uint64_t Cap);
  uint64_t Cap() const { return cap_; }
  // Queue this step's Extras and write this shard's block to Block (room for
  // 1 + Cap() words); returns the words written (1 + values sent).
  uint64_t Pack(const std::vector<uint64_t> &Extras, bool Done, uint64_t *Block);
  size_t Queued() const { return carry_.size() - head_; }
  // World blocks in rank order: each Stride words apart (0: packed back to
  // back, each 1 + its count words). All = every block's values in rank
  // order; AllDone = every block says done. false: a malformed block.
  static bool Unpack(const uint64_t *Blocks, size_t Words, uint64_t World, uint64_t Stride, uint64_t Cap,
                     std::vector<uint64_t> &All, bool *AllDone);

 private:
  uint64_t cap_;
  std::vector<uint64_t> carry_;  // queued values: [head_, size)
  size_t head_ = 0;
};

}  // namespace wtfgpu_host
