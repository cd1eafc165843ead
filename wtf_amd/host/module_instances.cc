// module_instances.cc — see module_instances.h.
#include "module_instances.h"

#include <dlfcn.h>
#include <fcntl.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>

namespace wtfgpu_host {

namespace {
thread_local ModuleInstances *t_registering = nullptr;

bool write_all(int fd, const std::vector<char> &b) {
  size_t off = 0;
  while (off < b.size()) {
    const ssize_t n = write(fd, b.data() + off, b.size() - off);
    if (n <= 0) return false;
    off += (size_t)n;
  }
  return true;
}
}  // namespace

ModuleInstances *ModuleInstances::Registering() { return t_registering; }

bool ModuleInstances::Load(const std::string &SoPath, const std::string &Name, uint32_t Count) {
  if (Count == 0 || Count > kMaxInstances) {
    printf("module instances: %u copies requested (1 .. %u)\n", Count, kMaxInstances);
    return false;
  }
  std::ifstream f(SoPath, std::ios::binary);
  const std::vector<char> image((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (image.empty()) {
    printf("module instances: cannot read %s\n", SoPath.c_str());
    return false;
  }
  // a distinct file per copy (the loader shares one handle between dlopens
  // of the same path or the same file); each is unlinked once loaded, its
  // mapping keeps it alive
  const char *tmp = getenv("TMPDIR");
  std::string dir = std::string(tmp && *tmp ? tmp : "/tmp") + "/wtf_module_XXXXXX";
  if (!mkdtemp(dir.data())) {
    printf("module instances: mkdtemp in %s failed\n", dir.c_str());
    return false;
  }
  auto &Reg = Targets_t::Instance().Targets;
  bool ok = true;
  for (uint32_t k = 0; ok && k < Count; k++) {
    const std::string path = dir + "/m" + std::to_string(k) + ".so";
    const int fd = open(path.c_str(), O_CREAT | O_WRONLY | O_TRUNC | O_CLOEXEC, 0700);
    ok = fd >= 0 && write_all(fd, image);
    if (fd >= 0) close(fd);
    const size_t before = Reg.size();
    void *h = ok ? dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL) : nullptr;
    unlink(path.c_str());
    if (!h) {
      printf("module instances: loading copy %u failed: %s\n", k, ok ? dlerror() : "write");
      ok = false;
      break;
    }
    handles_.push_back(h);
    const Target_t *T = nullptr;
    for (size_t i = before; i < Reg.size(); i++)
      if (Reg[i].Name == Name) T = &Reg[i];
    if (!T) {
      printf("module instances: %s registers no target named %s\n", SoPath.c_str(), Name.c_str());
      ok = false;
      break;
    }
    targets_.push_back(*T);
    Reg.erase(Reg.begin() + (std::ptrdiff_t)before, Reg.end());
  }
  rmdir(dir.c_str());
  if (!ok) return false;
  handlers_.assign(Count, {});
  return true;
}

bool ModuleInstances::InitAll(const Options_t &Opts, const CpuState_t &State) {
  for (uint32_t k = 0; k < Count(); k++) {
    t_registering = this;
    reg_ = (int)k;
    const bool ok = targets_[k].Init(Opts, State);
    t_registering = nullptr;
    reg_ = -1;
    if (!ok) {
      printf("module instances: Init of copy %u failed\n", k);
      return false;
    }
    if (k && handlers_[k].size() != handlers_[0].size()) {
      printf("module instances: copy %u hooked %zu rips, copy 0 %zu\n", k, handlers_[k].size(),
             handlers_[0].size());
      return false;
    }
  }
  return true;
}

void ModuleInstances::AddHandler(uint64_t Rip, BreakpointHandler_t Handler) { handlers_.at(reg_)[Rip] = Handler; }

BreakpointHandler_t ModuleInstances::HandlerOf(uint32_t Lane, uint64_t Rip) const {
  if (Lane >= handlers_.size()) return nullptr;
  const auto it = handlers_[Lane].find(Rip);
  return it == handlers_[Lane].end() ? nullptr : it->second;
}

}  // namespace wtfgpu_host
