// module_slots.cc — see module_slots.h.
#include "module_slots.h"

#include <dlfcn.h>
#include <link.h>

#include <cstdio>
#include <cstring>

namespace wtfgpu_host {

namespace {
struct FindCtx {
  const char *path;
  std::vector<std::pair<uintptr_t, size_t>> rw;
  std::pair<uintptr_t, size_t> relro{0, 0};
  bool found = false;
};

int find_module(struct dl_phdr_info *info, size_t, void *data) {
  FindCtx *c = (FindCtx *)data;
  if (!info->dlpi_name || !strstr(info->dlpi_name, c->path)) return 0;
  c->found = true;
  for (int i = 0; i < info->dlpi_phnum; i++) {
    const ElfW(Phdr) &ph = info->dlpi_phdr[i];
    const uintptr_t a = info->dlpi_addr + ph.p_vaddr;
    if (ph.p_type == PT_LOAD && (ph.p_flags & PF_W)) c->rw.push_back({a, ph.p_memsz});
    if (ph.p_type == PT_GNU_RELRO) c->relro = {a, ph.p_memsz};
  }
  return 1;
}
}  // namespace

bool ModuleSlots::Load(const std::string &so_path) {
  handle_ = dlopen(so_path.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!handle_) {
    fprintf(stderr, "ModuleSlots: dlopen(%s): %s\n", so_path.c_str(), dlerror());
    return false;
  }
  const char *base = strrchr(so_path.c_str(), '/');
  FindCtx c;
  c.path = base ? base + 1 : so_path.c_str();
  dl_iterate_phdr(find_module, &c);
  if (!c.found) return false;
  for (auto [a, n] : c.rw) {
    // drop the RELRO prefix (GOT / vtables made read-only after relocation)
    uintptr_t lo = a, hi = a + n;
    const uintptr_t rlo = c.relro.first, rhi = c.relro.first + c.relro.second;
    if (c.relro.second && rlo <= lo && rhi > lo) lo = rhi < hi ? rhi : hi;
    if (hi > lo) segs_.push_back({(uint8_t *)lo, hi - lo});
  }
  return true;
}

size_t ModuleSlots::StateBytes() const {
  size_t n = 0;
  for (auto &s : segs_) n += s.size;
  return n;
}

void ModuleSlots::Capture(uint32_t lanes) {
  initial_.resize(StateBytes());
  size_t off = 0;
  for (auto &s : segs_) {
    memcpy(initial_.data() + off, s.addr, s.size);
    off += s.size;
  }
  slots_.assign(lanes, {});
  touched_.assign(lanes, 0);
  in_ = -1;
}

void ModuleSlots::SwapIn(uint32_t lane) {
  const std::vector<uint8_t> &src = touched_[lane] ? slots_[lane] : initial_;
  size_t off = 0;
  for (auto &s : segs_) {
    memcpy(s.addr, src.data() + off, s.size);
    off += s.size;
  }
  in_ = (int32_t)lane;
}

void ModuleSlots::SwapOut(uint32_t lane) {
  std::vector<uint8_t> &dst = slots_[lane];
  dst.resize(initial_.size());
  size_t off = 0;
  for (auto &s : segs_) {
    memcpy(dst.data() + off, s.addr, s.size);
    off += s.size;
  }
  touched_[lane] = 1;
  in_ = -1;
}

}  // namespace wtfgpu_host
