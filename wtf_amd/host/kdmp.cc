// kdmp.cc — see kdmp.h. Header offsets from kdmp-parser-structs.h:558-674.
#include "kdmp.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>

namespace wtfgpu_host {

namespace {
constexpr uint32_t kSigPage = 0x45474150;   // 'PAGE'
constexpr uint32_t kValidDu64 = 0x34365544; // 'DU64'
constexpr uint64_t kOffDtb = 0x10, kOffPhysmem = 0x88, kOffContext = 0x348, kOffDumpType = 0xf98, kOffBmp = 0x2000;
constexpr uint32_t kFullDump = 1, kBmpDump = 5;
constexpr uint32_t kBmpSigS = 0x504d4453, kBmpSigF = 0x504d4446, kBmpValid = 0x504d5544;

template <typename T>
T rd(const uint8_t *p) {
  T v;
  memcpy(&v, p, sizeof(T));
  return v;
}
}  // namespace

KernelDump::~KernelDump() {
  if (map_) munmap(map_, size_);
}

bool KernelDump::Parse(const std::string &path) {
  const int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < (off_t)kOffBmp) {
    close(fd);
    return false;
  }
  size_ = (size_t)st.st_size;
  void *m = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (m == MAP_FAILED) return false;
  map_ = (uint8_t *)m;
  const uint8_t *h = map_;
  if (rd<uint32_t>(h) != kSigPage || rd<uint32_t>(h + 4) != kValidDu64) return false;
  dtb_ = rd<uint64_t>(h + kOffDtb);
  rip_ = rd<uint64_t>(h + kOffContext + 0xf8);  // CONTEXT.Rip
  dump_type_ = rd<uint32_t>(h + kOffDumpType);
  if (dump_type_ == kFullDump) {
    const uint32_t nruns = rd<uint32_t>(h + kOffPhysmem);
    uint64_t off = kOffBmp;
    for (uint32_t r = 0; r < nruns; r++) {
      const uint8_t *run = h + kOffPhysmem + 0x10 + 16ull * r;
      if ((size_t)(run - h) + 16 > kOffBmp) return false;
      const uint64_t base = rd<uint64_t>(run), count = rd<uint64_t>(run + 8);
      for (uint64_t i = 0; i < count; i++, off += 0x1000) {
        if (off + 0x1000 > size_) return false;
        pages_.try_emplace(base + i, map_ + off);
      }
    }
    return true;
  }
  if (dump_type_ == kBmpDump) {
    const uint8_t *b = h + kOffBmp;
    const uint32_t sig = rd<uint32_t>(b), valid = rd<uint32_t>(b + 4);
    if ((sig != kBmpSigS && sig != kBmpSigF) || valid != kBmpValid) return false;
    const uint64_t first = rd<uint64_t>(b + 0x20), npages = rd<uint64_t>(b + 0x30);
    const uint8_t *bitmap = b + 0x38;
    uint64_t off = first;
    for (uint64_t byte = 0; byte < npages / 8; byte++) {
      if ((size_t)(bitmap + byte - h) >= size_) return false;
      const uint8_t v = bitmap[byte];
      for (int bit = 0; bit < 8; bit++) {
        if (!((v >> bit) & 1)) continue;
        if (off + 0x1000 > size_) return false;
        pages_.try_emplace(byte * 8 + bit, map_ + off);
        off += 0x1000;
      }
    }
    return true;
  }
  return false;
}

const uint8_t *KernelDump::GetPhysicalPage(uint64_t gpa) const {
  auto it = pages_.find(gpa >> 12);
  return it == pages_.end() ? nullptr : it->second;
}

std::optional<uint64_t> KernelDump::VirtTranslate(uint64_t gva, uint64_t dtb) const {
  uint64_t table = (dtb ? dtb : dtb_) & 0x000ffffffffff000ull;
  for (int level = 3; level >= 0; level--) {
    const uint8_t *pg = GetPhysicalPage(table);
    if (!pg) return std::nullopt;
    const uint64_t e = rd<uint64_t>(pg + ((gva >> (12 + 9 * level)) & 0x1ff) * 8);
    if (!(e & 1)) return std::nullopt;
    const uint64_t frame = e & 0x000ffffffffff000ull;
    if (level == 2 && (e & 0x80)) return (frame & ~0x3fffffffull) | (gva & 0x3fffffffull);
    if (level == 1 && (e & 0x80)) return (frame & ~0x1fffffull) | (gva & 0x1fffffull);
    table = frame;
  }
  return table | (gva & 0xfff);
}

std::vector<std::pair<uint64_t, const uint8_t *>> KernelDump::Pages() const {
  std::vector<std::pair<uint64_t, const uint8_t *>> v(pages_.begin(), pages_.end());
  std::sort(v.begin(), v.end(), [](auto &a, auto &b) { return a.first < b.first; });
  return v;
}

std::vector<uint64_t> ExecutablePages(const KernelDump &Dump, uint64_t cr3, size_t max_pages) {
  std::vector<uint64_t> vpns;
  const uint64_t mask = 0x000ffffffffff000ull;
  auto entry = [&](uint64_t table, uint64_t idx, uint64_t &e) {
    const uint8_t *pg = Dump.GetPhysicalPage(table & mask);
    if (!pg) return false;
    memcpy(&e, pg + idx * 8, 8);
    return (e & 1) != 0;
  };
  cr3 &= mask;
  for (uint64_t i4 = 0; i4 < 512 && vpns.size() < max_pages; i4++) {
    uint64_t e4;
    if (!entry(cr3, i4, e4)) continue;
    for (uint64_t i3 = 0; i3 < 512 && vpns.size() < max_pages; i3++) {
      uint64_t e3;
      if (!entry(e4, i3, e3)) continue;
      const bool nx3 = ((e4 | e3) >> 63) & 1;
      if (e3 & 0x80) continue;
      for (uint64_t i2 = 0; i2 < 512 && vpns.size() < max_pages; i2++) {
        uint64_t e2;
        if (!entry(e3, i2, e2)) continue;
        const bool nx2 = nx3 || ((e2 >> 63) & 1);
        uint64_t va = (i4 << 39) | (i3 << 30) | (i2 << 21);
        if (va & (1ull << 47)) va |= 0xffff000000000000ull;
        if (e2 & 0x80) {
          if (!nx2)
            for (uint64_t k = 0; k < 512; k++) vpns.push_back((va >> 12) + k);
          continue;
        }
        for (uint64_t i1 = 0; i1 < 512 && vpns.size() < max_pages; i1++) {
          uint64_t e1;
          if (!entry(e2, i1, e1)) continue;
          if (nx2 || ((e1 >> 63) & 1)) continue;
          vpns.push_back((va >> 12) + i1);
        }
      }
    }
  }
  return vpns;
}

}  // namespace wtfgpu_host
