// gpu_backend.cc — see gpu_backend.h. Reference functions are cited per method.
#include "gpu_backend.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>

#include "blake3_lite.h"

namespace wtfgpu_host {

namespace {
using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

// Registers_t -> index in the 18-u64 gpr view (wtfgpu order), -1 = not a gpr
int gpr_index(Registers_t r) {
  switch (r) {
    case Registers_t::Rax: return WTFGPU_RAX;
    case Registers_t::Rbx: return WTFGPU_RBX;
    case Registers_t::Rcx: return WTFGPU_RCX;
    case Registers_t::Rdx: return WTFGPU_RDX;
    case Registers_t::Rsi: return WTFGPU_RSI;
    case Registers_t::Rdi: return WTFGPU_RDI;
    case Registers_t::Rsp: return WTFGPU_RSP;
    case Registers_t::Rbp: return WTFGPU_RBP;
    case Registers_t::R8: return WTFGPU_R8;
    case Registers_t::R9: return WTFGPU_R9;
    case Registers_t::R10: return WTFGPU_R10;
    case Registers_t::R11: return WTFGPU_R11;
    case Registers_t::R12: return WTFGPU_R12;
    case Registers_t::R13: return WTFGPU_R13;
    case Registers_t::R14: return WTFGPU_R14;
    case Registers_t::R15: return WTFGPU_R15;
    case Registers_t::Rip: return 16;
    case Registers_t::Rflags: return 17;
    default: return -1;
  }
}

}  // namespace

GpuBackend_t::GpuBackend_t() = default;
GpuBackend_t::~GpuBackend_t() {
  if (ctx_) wtfgpu_destroy(ctx_);
}

bool GpuBackend_t::LoadDump(const std::string &dump_path) { return dump_.Parse(dump_path); }

// bochscpu_backend.cc:269-335: the dump becomes the device page pool
bool GpuBackend_t::Initialize(const Options_t &Opts, const CpuState_t &CpuState) {
  if (dump_.PageCount() == 0 && !Opts.DumpPath.empty() && !LoadDump(Opts.DumpPath.string())) {
    printf("Failed to parse the dump %s\n", Opts.DumpPath.string().c_str());
    return false;
  }
  if (wtfgpu_create(Opts.GpuDevice, &ctx_) != WTFGPU_OK) {
    printf("wtfgpu_create(%d) failed\n", Opts.GpuDevice);
    return false;
  }
  const auto pages = dump_.Pages();
  std::vector<uint64_t> gpfns(pages.size());
  std::vector<uint8_t> blob(pages.size() * Page::Size);
  for (size_t i = 0; i < pages.size(); i++) {
    gpfns[i] = pages[i].first;
    memcpy(blob.data() + i * Page::Size, pages[i].second, Page::Size);
  }
  if (wtfgpu_load_pool(ctx_, gpfns.data(), blob.data(), gpfns.size())) return false;
  nlanes_ = std::max<uint32_t>(Opts.GpuLanes, 1);
  overlay_pages_ = std::max<uint32_t>(Opts.GpuOverlayPages, 1);
  if (wtfgpu_alloc_lanes(ctx_, nlanes_, overlay_pages_, 1024)) return false;
  views_.clear();
  views_.resize(nlanes_);
  if (Opts.Limit) SetLimit(Opts.Limit);
  if (!Restore(CpuState)) return false;
  return set_code_pages();
}

// bochscpu_backend.cc:730-797 (+ LoadState :1026-1122): registers from the
// state, dirty overlays dropped on the device, result back to Ok.
bool GpuBackend_t::Restore(const CpuState_t &CpuState) {
  initial_ = CpuState;
  initial_regs_ = RegsFromCpuState(CpuState);
  if (wtfgpu_set_initial_state(ctx_, &initial_regs_)) return false;
  if (wtfgpu_restore(ctx_, 0, nlanes_)) return false;
  for (uint32_t l = 0; l < nlanes_; l++) reset_view(l);
  cur_ = 0;
  return true;
}

void GpuBackend_t::reset_view(uint32_t lane) {
  LaneView &v = views_[lane];
  memcpy(v.gpr, initial_regs_.gpr, sizeof(initial_regs_.gpr));
  v.gpr[16] = initial_regs_.rip;
  v.gpr[17] = initial_regs_.rflags;
  v.regs_dirty = false;
  v.result.reset();
  v.seed = initial_.Seed;  // Rdrand seed (bochscpu_backend.cc:1030)
  v.dirty_known = true;    // a restored lane has an empty overlay
  v.dirty.clear();
  v.pages.clear();
}

void GpuBackend_t::Stop(const TestcaseResult_t &Res) { cur().result = Res; }

void GpuBackend_t::SetLimit(const uint64_t Limit) {
  limit_ = Limit;
  if (ctx_) wtfgpu_set_limit(ctx_, Limit);
}

uint64_t GpuBackend_t::GetReg(const Registers_t Reg) {
  const int i = gpr_index(Reg);
  if (i >= 0) return cur().gpr[i];
  if (Reg == Registers_t::Cr3) return initial_.Cr3;  // ring-3 lanes cannot change cr3
  if (Reg == Registers_t::Cr2) return initial_.Cr2;
  return 0;
}

uint64_t GpuBackend_t::SetReg(const Registers_t Reg, const uint64_t Value) {
  const int i = gpr_index(Reg);
  if (i >= 0) {
    cur().gpr[i] = Value;
    cur().regs_dirty = true;
  }
  return Value;
}

// bochscpu_backend.cc:874-885, per-lane seed
uint64_t GpuBackend_t::Rdrand() { return wtf_rdrand(cur().seed); }

void GpuBackend_t::PrintRunStats() {
  printf("--------------------------------------------------\n");
  printf("Run stats (gpu):\n");
  printf("Instructions executed: %llu\n", (unsigned long long)stats_.retired);
  printf("  Breakpoint services: %llu in %llu rounds\n", (unsigned long long)stats_.breakpoint_hits,
         (unsigned long long)stats_.rounds);
  printf("       Kernel time ms: %.2f\n", stats_.kernel_ms);
}

// bochscpu_backend.cc:337-346
bool GpuBackend_t::SetBreakpoint(const Gva_t Gva, const BreakpointHandler_t Handler) {
  if (breakpoints_.count(Gva.U64())) {
    printf("/!\\ There is already a breakpoint at %#llx\n", (unsigned long long)Gva.U64());
    return false;
  }
  breakpoints_.emplace(Gva.U64(), Handler);
  std::vector<uint64_t> v;
  for (auto &kv : breakpoints_) v.push_back(kv.first);
  return wtfgpu_set_breakpoints(ctx_, v.data(), (uint32_t)v.size()) == WTFGPU_OK;
}

// Writes go to lane overlays, which the device dirties by itself.
bool GpuBackend_t::DirtyGpa(const Gpa_t) { return true; }

// The lane's view of a physical page, on the host: staged copy, else a fetch of
// the lane's overlay page, else the dump page (or zeros).
uint8_t *GpuBackend_t::lane_page(uint32_t lane, uint64_t gpfn) const {
  LaneView &v = views_[lane];
  auto it = v.pages.find(gpfn);
  if (it != v.pages.end()) return it->second.data.get();
  if (!v.dirty_known) {
    std::vector<uint32_t> buf(overlay_pages_ + 1);
    wtfgpu_read_dirty_list(ctx_, &lane, 1, buf.data());
    v.dirty.assign(buf.begin() + 1, buf.begin() + 1 + std::min<uint32_t>(buf[0], overlay_pages_));
    v.dirty_known = true;
  }
  HostPage hp;
  hp.data.reset(new uint8_t[Page::Size]);
  const bool in_overlay = std::find(v.dirty.begin(), v.dirty.end(), (uint32_t)gpfn) != v.dirty.end();
  if (in_overlay) {
    const uint64_t gpa = gpfn << 12;
    wtfgpu_gather_pages(ctx_, &lane, &gpa, 1, hp.data.get());
    stats_.page_fetches++;
  } else if (const uint8_t *p = dump_.GetPhysicalPage(gpfn << 12)) {
    memcpy(hp.data.get(), p, Page::Size);
  } else {
    memset(hp.data.get(), 0, Page::Size);
  }
  hp.orig.reset(new uint8_t[Page::Size]);
  memcpy(hp.orig.get(), hp.data.get(), Page::Size);
  uint8_t *r = hp.data.get();
  v.pages.emplace(gpfn, std::move(hp));
  return r;
}

// bochscpu_mem_virt_translate semantics (present bits only), on the lane view
bool GpuBackend_t::VirtTranslate(const Gva_t Gva, Gpa_t &Gpa, const MemoryValidate_t) const {
  uint64_t table = initial_.Cr3 & 0x000ffffffffff000ull;
  const uint64_t va = Gva.U64();
  for (int level = 3; level >= 0; level--) {
    const uint8_t *pg = lane_page(cur_, table >> 12);
    uint64_t e;
    memcpy(&e, pg + ((va >> (12 + 9 * level)) & 0x1ff) * 8, 8);
    if (!(e & 1)) return false;
    const uint64_t frame = e & 0x000ffffffffff000ull;
    if (level == 2 && (e & 0x80)) {
      Gpa = Gpa_t((frame & ~0x3fffffffull) | (va & 0x3fffffffull));
      return true;
    }
    if (level == 1 && (e & 0x80)) {
      Gpa = Gpa_t((frame & ~0x1fffffull) | (va & 0x1fffffull));
      return true;
    }
    table = frame;
  }
  Gpa = Gpa_t(table | (va & 0xfff));
  return true;
}

// A host pointer into the lane's staged copy of the page: writes through it are
// diffed against the original at flush time and applied to the lane overlay.
uint8_t *GpuBackend_t::PhysTranslate(const Gpa_t Gpa) const {
  return lane_page(cur_, Gpa.U64() >> 12) + (Gpa.U64() & 0xfff);
}

bool GpuBackend_t::PageFaultsMemoryIfNeeded(const Gva_t, const uint64_t) {
  // needs #PF injection through the guest IDT: not in this engine yet
  return false;
}

const std::unordered_set<Gva_t> &GpuBackend_t::LastNewCoverage() const { return last_new_coverage_; }

// bochscpu_backend.cc:1005-1016
bool GpuBackend_t::RevokeLastNewCoverage() {
  for (const Gva_t &g : last_new_coverage_) aggregate_.erase(g.U64());
  last_new_coverage_.clear();
  return true;
}

// Staged registers and memory of `lanes` -> device.
int GpuBackend_t::flush_lanes(const std::vector<uint32_t> &lanes) {
  std::vector<uint32_t> rl;
  std::vector<uint64_t> regs;
  std::vector<wtfgpu_write_t> writes;
  std::vector<uint8_t> data;
  for (uint32_t l : lanes) {
    LaneView &v = views_[l];
    if (v.regs_dirty) {
      rl.push_back(l);
      regs.insert(regs.end(), v.gpr, v.gpr + 18);
      v.regs_dirty = false;
    }
    for (auto &[gpfn, hp] : v.pages) {
      size_t lo = 0, hi = Page::Size;
      while (lo < hi && hp.data[lo] == hp.orig[lo]) lo++;
      while (hi > lo && hp.data[hi - 1] == hp.orig[hi - 1]) hi--;
      if (lo == hi) continue;
      wtfgpu_write_t w{};
      w.lane = l;
      w.len = (uint32_t)(hi - lo);
      w.gva = (gpfn << 12) | lo;
      w.data_off = data.size();
      data.insert(data.end(), hp.data.get() + lo, hp.data.get() + hi);
      writes.push_back(w);
      v.dirty_known = false;  // the device overlay changed
    }
    v.pages.clear();
  }
  int rc = WTFGPU_OK;
  if (!rl.empty()) rc = wtfgpu_write_gprs_list(ctx_, rl.data(), (uint32_t)rl.size(), regs.data());
  if (!rc && !writes.empty())
    rc = wtfgpu_apply_phys_writes(ctx_, writes.data(), (uint32_t)writes.size(), data.data(), data.size(), nullptr);
  return rc;
}

// The run loop over `lanes` (ascending): launch, classify exits, service
// breakpoint hits on the host, resume; until every lane has a result.
bool GpuBackend_t::run_lanes(const std::vector<uint32_t> &lanes, std::vector<LaneResult> *out, ModuleSlots *slots,
                             bool per_lane_state) {
  if (lanes.empty()) return true;
  const uint32_t first = lanes.front() & ~63u, count = lanes.back() + 1 - first;
  const uint32_t cpl = initial_.Cs.Selector & 3;
  std::vector<wtfgpu_exit_t> ex(count);
  std::vector<uint8_t> done(count, 0);
  std::vector<uint32_t> pending = lanes;
  // lanes stopped before running (InsertTestcase called Stop)
  std::vector<uint32_t> pre_stopped;
  for (uint32_t l : lanes)
    if (views_[l].result) pre_stopped.push_back(l);
  if (!pre_stopped.empty()) wtfgpu_stop(ctx_, pre_stopped.data(), (uint32_t)pre_stopped.size(), WTFGPU_EXIT_STOPPED);
  for (uint32_t l : pre_stopped) done[l - first] = 1;

  for (;;) {
    wtfgpu_run_stats_t rs{};
    if (wtfgpu_run(ctx_, first, count, ~0ull, &rs)) return false;
    stats_.kernel_launches += rs.kernel_launches;
    stats_.kernel_ms += rs.kernel_ms;
    stats_.retired += rs.lane_retired;
    stats_.rounds++;
    if (wtfgpu_read_exits(ctx_, first, count, ex.data())) return false;
    const auto t0 = Clock::now();
    std::vector<uint32_t> hits;
    for (uint32_t l : pending) {
      if (done[l - first]) continue;
      const wtfgpu_exit_t &e = ex[l - first];
      LaneView &v = views_[l];
      switch (e.status) {
        case WTFGPU_EXIT_BREAKPOINT: hits.push_back(l); continue;
        case WTFGPU_EXIT_TIMEOUT: v.result = Timedout_t(); break;    // bochscpu_backend.cc:458-469
        case WTFGPU_EXIT_INT3:                                         // :595-619
        case WTFGPU_EXIT_HLT: v.result = Crash_t(); break;             // :690-697
        case WTFGPU_EXIT_CR3: v.result = Cr3Change_t(); break;         // :628-657
        case WTFGPU_EXIT_FAULT: v.result = FaultToResult(e.vector, e.error, e.rip, cpl); break;
        case WTFGPU_EXIT_STOPPED: break;
        default:  // unimplemented opcode / overlay full: the engine cannot finish it
          if (out) (*out)[l].error = true;
          if (!v.result) v.result = Crash_t("engine-" + std::to_string(e.status));
          break;
      }
      done[l - first] = 1;
    }
    if (hits.empty()) break;
    // ---- service the round's breakpoint hits
    std::vector<uint64_t> regs(hits.size() * 18);
    if (wtfgpu_read_gprs_list(ctx_, hits.data(), (uint32_t)hits.size(), regs.data())) return false;
    const uint32_t stride = overlay_pages_ + 1;
    std::vector<uint32_t> dl(hits.size() * stride);
    if (wtfgpu_read_dirty_list(ctx_, hits.data(), (uint32_t)hits.size(), dl.data())) return false;
    // prefetch the stack page of every hit lane whose overlay holds it (handlers
    // read their return address / arguments there)
    std::vector<uint32_t> pf_lanes;
    std::vector<uint64_t> pf_gpas;
    for (size_t i = 0; i < hits.size(); i++) {
      LaneView &v = views_[hits[i]];
      memcpy(v.gpr, &regs[i * 18], 18 * 8);
      v.regs_dirty = false;
      v.pages.clear();
      const uint32_t cnt = std::min(dl[i * stride], overlay_pages_);
      v.dirty.assign(dl.begin() + i * stride + 1, dl.begin() + i * stride + 1 + cnt);
      v.dirty_known = true;
      cur_ = hits[i];
      Gpa_t sp;
      if (VirtTranslate(Gva_t(v.gpr[WTFGPU_RSP]), sp, MemoryValidate_t::ValidateRead) &&
          std::find(v.dirty.begin(), v.dirty.end(), (uint32_t)(sp.U64() >> 12)) != v.dirty.end()) {
        pf_lanes.push_back(hits[i]);
        pf_gpas.push_back(sp.U64() & ~0xfffull);
      }
    }
    if (!pf_lanes.empty()) {
      std::vector<uint8_t> buf(pf_lanes.size() * Page::Size);
      if (wtfgpu_gather_pages(ctx_, pf_lanes.data(), pf_gpas.data(), (uint32_t)pf_lanes.size(), buf.data()))
        return false;
      for (size_t i = 0; i < pf_lanes.size(); i++) {
        HostPage hp;
        hp.data.reset(new uint8_t[Page::Size]);
        hp.orig.reset(new uint8_t[Page::Size]);
        memcpy(hp.data.get(), buf.data() + i * Page::Size, Page::Size);
        memcpy(hp.orig.get(), hp.data.get(), Page::Size);
        views_[pf_lanes[i]].pages[pf_gpas[i] >> 12] = std::move(hp);
      }
      stats_.prefetched_pages += pf_lanes.size();
    }
    std::vector<uint32_t> resume, stop;
    std::vector<uint8_t> skip;
    Backend_t *saved = g_Backend;
    g_Backend = this;
    for (uint32_t l : hits) {
      LaneView &v = views_[l];
      cur_ = l;
      const uint64_t rip0 = v.gpr[16];
      auto it = breakpoints_.find(rip0);
      if (per_lane_state && slots) slots->SwapIn(l);
      if (it != breakpoints_.end()) it->second(this);  // BeforeExecutionHook (bochscpu_backend.cc:545-547)
      if (per_lane_state && slots) slots->SwapOut(l);
      stats_.breakpoint_hits++;
      if (v.result) {
        stop.push_back(l);
        done[l - first] = 1;
      } else {
        resume.push_back(l);
        skip.push_back(v.gpr[16] == rip0 ? 1 : 0);  // U10: a moved rip cancels the hooked instruction
      }
    }
    g_Backend = saved;
    if (flush_lanes(hits)) return false;
    if (!stop.empty() && wtfgpu_stop(ctx_, stop.data(), (uint32_t)stop.size(), WTFGPU_EXIT_STOPPED)) return false;
    if (!resume.empty() && wtfgpu_resume(ctx_, resume.data(), (uint32_t)resume.size(), skip.data())) return false;
    stats_.service_ms += ms_since(t0);
    pending = resume;
  }
  // final state of every lane
  if (out) {
    std::vector<uint64_t> regs(lanes.size() * 18);
    if (wtfgpu_read_gprs_list(ctx_, lanes.data(), (uint32_t)lanes.size(), regs.data())) return false;
    if (wtfgpu_read_exits(ctx_, first, count, ex.data())) return false;
    for (size_t i = 0; i < lanes.size(); i++) {
      LaneResult &r = (*out)[lanes[i]];
      const LaneView &v = views_[lanes[i]];
      r.result = v.result ? *v.result : TestcaseResult_t(Ok_t());
      memcpy(r.gprs, &regs[i * 18], 18 * 8);
      r.rip = r.gprs[16];
      r.icount = ex[lanes[i] - first].icount;
      r.exit_status = ex[lanes[i] - first].status;
    }
  }
  return true;
}

// Per-lane new rips, attributed in lane order against the aggregate set
// (bochscpu_backend.cc:501-504); timed-out lanes have theirs revoked
// (client.cc:122-125); the new rips join the device coverage map.
void GpuBackend_t::finish_coverage(uint32_t n, std::vector<LaneResult> *out, std::vector<uint32_t> *timedout) {
  uint64_t total = 0;
  uint32_t ovf = 0, dl = 0;
  uint64_t dr = 0;
  wtfgpu_read_coverage(ctx_, 0, n, &dl, &dr, 0, &total, &ovf);
  std::vector<uint32_t> lanes(total);
  std::vector<uint64_t> rips(total);
  if (total) wtfgpu_read_coverage(ctx_, 0, n, lanes.data(), rips.data(), total, &total, &ovf);
  std::vector<std::vector<uint64_t>> per(n);
  for (uint64_t i = 0; i < total; i++) per[lanes[i]].push_back(rips[i]);
  std::vector<uint64_t> fresh;
  last_new_coverage_.clear();
  for (uint32_t l = 0; l < n; l++) {
    std::sort(per[l].begin(), per[l].end());
    per[l].erase(std::unique(per[l].begin(), per[l].end()), per[l].end());
    if (full_coverage_) {
      if (out) (*out)[l].new_coverage = per[l];
      continue;
    }
    const bool revoke = timedout && std::find(timedout->begin(), timedout->end(), l) != timedout->end();
    for (uint64_t rip : per[l]) {
      if (aggregate_.count(rip)) continue;
      if (out) (*out)[l].new_coverage.push_back(rip);
      if (revoke) continue;
      aggregate_.insert(rip);
      fresh.push_back(rip);
      if (n == 1) last_new_coverage_.insert(Gva_t(rip));
    }
  }
  if (full_coverage_) {  // parity mode: every lane ran against an empty map
    wtfgpu_reset_coverage(ctx_);
    return;
  }
  if (!fresh.empty()) wtfgpu_commit_coverage(ctx_, fresh.data(), fresh.size());
}

// bochscpu_backend.cc:352-410: one testcase on lane 0; the caller already ran
// Target.InsertTestcase against this backend (client.cc:102-111).
std::optional<TestcaseResult_t> GpuBackend_t::Run(const uint8_t *, const uint64_t) {
  const auto t0 = Clock::now();
  cur_ = 0;
  if (flush_lanes({0})) return std::nullopt;
  std::vector<LaneResult> out(1);
  if (!run_lanes({0}, &out, nullptr, false)) return std::nullopt;
  std::vector<uint32_t> to;
  if (std::holds_alternative<Timedout_t>(out[0].result)) to.push_back(0);
  finish_coverage(1, nullptr, nullptr);  // Timedout revocation is the client's call (RevokeLastNewCoverage)
  stats_.total_ms += ms_since(t0);
  cur_ = 0;
  return out[0].result;
}

bool GpuBackend_t::RunBatch(const Target_t &Target, const std::vector<std::pair<const uint8_t *, size_t>> &Testcases,
                            std::vector<LaneResult> &Out, ModuleSlots *Slots) {
  const auto t0 = Clock::now();
  const uint32_t n = (uint32_t)Testcases.size();
  if (n == 0 || n > nlanes_) return false;
  Out.assign(n, LaneResult{});
  if (Slots) Slots->ResetAll();
  if (wtfgpu_restore(ctx_, 0, n)) return false;
  for (uint32_t l = 0; l < n; l++) reset_view(l);
  // InsertTestcase per lane (client.cc:102), module state per lane
  Backend_t *saved = g_Backend;
  g_Backend = this;
  std::vector<uint32_t> lanes(n);
  for (uint32_t l = 0; l < n; l++) {
    lanes[l] = l;
    cur_ = l;
    if (Slots) Slots->SwapIn(l);
    const bool ok = Target.InsertTestcase(Testcases[l].first, Testcases[l].second);
    if (Slots) Slots->SwapOut(l);
    if (!ok) views_[l].result = Crash_t("insert-testcase-failed");
  }
  g_Backend = saved;
  if (flush_lanes(lanes)) return false;
  if (!run_lanes(lanes, &Out, Slots, Slots != nullptr)) return false;
  std::vector<uint32_t> timedout;
  for (uint32_t l = 0; l < n; l++)
    if (std::holds_alternative<Timedout_t>(Out[l].result)) timedout.push_back(l);
  finish_coverage(n, &Out, &timedout);
  // Target.Restore per lane (client.cc:145), then the device restore happens
  // at the start of the next batch (dirty-list reset)
  g_Backend = this;
  for (uint32_t l = 0; l < n; l++) {
    cur_ = l;
    if (Slots) Slots->SwapIn(l);
    Target.Restore();
    if (Slots) Slots->SwapOut(l);
  }
  g_Backend = saved;
  cur_ = 0;
  stats_.total_ms += ms_since(t0);
  stats_.batches++;
  stats_.testcases += n;
  return true;
}

void GpuBackend_t::ResetCoverage() {
  aggregate_.clear();
  last_new_coverage_.clear();
  wtfgpu_reset_coverage(ctx_);
}

std::string GpuBackend_t::StatsJson() const {
  char b[512];
  snprintf(b, sizeof(b),
           "{\"kind\":\"gpu\",\"rounds\":%llu,\"breakpoint_hits\":%llu,\"kernel_launches\":%llu,"
           "\"kernel_ms\":%.3f,\"service_ms\":%.3f,\"total_ms\":%.3f,\"page_fetches\":%llu,"
           "\"prefetched_pages\":%llu}",
           (unsigned long long)stats_.rounds, (unsigned long long)stats_.breakpoint_hits,
           (unsigned long long)stats_.kernel_launches, stats_.kernel_ms, stats_.service_ms, stats_.total_ms,
           (unsigned long long)stats_.page_fetches, (unsigned long long)stats_.prefetched_pages);
  return b;
}

// Coverage index space: every executable leaf page reachable
// from the snapshot cr3 gets a slot in the device coverage map; identical on
// every GPU, so the maps can be merged with a MAX all-reduce.
bool GpuBackend_t::set_code_pages() {
  std::vector<uint64_t> vpns;
  const uint64_t kMaxPages = 1u << 16;
  const uint64_t mask = 0x000ffffffffff000ull;
  auto entry = [&](uint64_t table, uint64_t idx, uint64_t &e) {
    const uint8_t *pg = dump_.GetPhysicalPage(table & mask);
    if (!pg) return false;
    memcpy(&e, pg + idx * 8, 8);
    return (e & 1) != 0;
  };
  const uint64_t cr3 = initial_.Cr3 & mask;
  for (uint64_t i4 = 0; i4 < 512 && vpns.size() < kMaxPages; i4++) {
    uint64_t e4;
    if (!entry(cr3, i4, e4)) continue;
    for (uint64_t i3 = 0; i3 < 512 && vpns.size() < kMaxPages; i3++) {
      uint64_t e3;
      if (!entry(e4, i3, e3)) continue;
      const bool nx3 = ((e4 | e3) >> 63) & 1;
      if (e3 & 0x80) continue;  // 1 GiB leaves are data mappings in practice
      for (uint64_t i2 = 0; i2 < 512 && vpns.size() < kMaxPages; i2++) {
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
        for (uint64_t i1 = 0; i1 < 512 && vpns.size() < kMaxPages; i1++) {
          uint64_t e1;
          if (!entry(e2, i1, e1)) continue;
          if (nx2 || ((e1 >> 63) & 1)) continue;
          vpns.push_back((va >> 12) + i1);
        }
      }
    }
  }
  if (vpns.empty()) return true;
  return wtfgpu_set_code_pages(ctx_, vpns.data(), (uint32_t)vpns.size()) == WTFGPU_OK;
}

}  // namespace wtfgpu_host
