// kdmp.h — reader for the Windows kernel crash-dump files wtf snapshots ship as
// mem.dmp (64-bit full dumps and BMP dumps). Restates what the vendored
// kdmp-parser provides to the backend: the header checks, the GPA -> page map
// (full dump: pages from file offset 0x2000, run after run, kdmp-parser.h:399-484;
// BMP dump: FirstPage + bitmap, :490-529; first mapping of a GPA wins like its
// try_emplace), GetPhysicalPage (:233-254) and the 4-level VirtTranslate
// (:269-345, 1 GiB / 2 MiB leaves, no permission checks).
#pragma once
#include <cstdint>
#include <optional>
#include <string>
#include <unordered_map>
#include <vector>

namespace wtfgpu_host {

class KernelDump {
 public:
  ~KernelDump();
  bool Parse(const std::string &path);
  uint32_t DumpType() const { return dump_type_; }
  uint64_t DirectoryTableBase() const { return dtb_; }
  uint64_t ContextRip() const { return rip_; }
  // nullptr when the page is not in the dump (the backend reads it as zeros)
  const uint8_t *GetPhysicalPage(uint64_t gpa) const;
  std::optional<uint64_t> VirtTranslate(uint64_t gva, uint64_t dtb = 0) const;
  // every page, gpfn ascending
  std::vector<std::pair<uint64_t, const uint8_t *>> Pages() const;
  size_t PageCount() const { return pages_.size(); }

 private:
  uint8_t *map_ = nullptr;
  size_t size_ = 0;
  uint32_t dump_type_ = 0;
  uint64_t dtb_ = 0, rip_ = 0;
  std::unordered_map<uint64_t, const uint8_t *> pages_;  // gpfn -> page
};

// The coverage index space: every executable 4 KiB page (leaf
// not NX at any level) reachable from `cr3` in the dump, in page-table walk
// order, up to `max_pages`. 1 GiB leaves are skipped (data mappings in
// practice). Identical for every shard built from the same snapshot, so
// per-shard coverage maps over these slots merge with a MAX all-reduce.
std::vector<uint64_t> ExecutablePages(const KernelDump &Dump, uint64_t cr3, size_t max_pages = 1u << 16);

}  // namespace wtfgpu_host
