// gpu_backend.cc — see gpu_backend.h. Reference functions are cited per method.
#include "gpu_backend.h"
#include "module_instances.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>

#include "host_pool.h"

#include "blake3_lite.h"

namespace wtfgpu_host {

thread_local uint32_t GpuBackend_t::cur_ = 0;
thread_local uint64_t GpuBackend_t::servicing_bp_ = ~0ull;
thread_local uint64_t GpuBackend_t::servicing_sp_ = ~0ull;
thread_local bool GpuBackend_t::scouting_ = false;

namespace {
constexpr uint64_t kFeedRegion = 16384;  // engine.hip wtfgpu_set_feed_lanes per-lane region
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
  for (Part &P : parts_)
    for (void *p : {(void *)P.pin, (void *)P.ex, (void *)P.nb, (void *)P.dc, (void *)P.sargs, (void *)P.cov_hdr})
      if (p) wtfgpu_host_free(ctx_, p);
  if (wpin_) wtfgpu_host_free(ctx_, wpin_);
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
  if (wtfgpu_alloc_lanes(ctx_, nlanes_, overlay_pages_, Opts.GpuCoverageSet)) return false;
  views_.clear();
  views_.resize(nlanes_);
  touched_.assign(nlanes_, 0);
  pf_.assign(nlanes_, PrepFeed{});
  arenas_.resize(HostPool::Get().Threads() + 1);
  if (Opts.Limit) SetLimit(Opts.Limit);
  if (Opts.Edges && wtfgpu_set_edges(ctx_, 1) != WTFGPU_OK) return false;  // bochscpu_backend.cc:308-312
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
  v.cr[0] = initial_regs_.cr2;
  v.cr[1] = initial_regs_.cr3;
  v.cr_known = 3;
  v.cr_dirty = 0;
  v.result.reset();
  v.handler_fault = false;
  v.seed = initial_.Seed;  // Rdrand seed (bochscpu_backend.cc:1030)
  v.has_feed = false;
  v.feed.clear();
  v.dirty_known = true;    // a restored lane has an empty overlay
  v.dirty.clear();
  v.wlog.clear();
  v.wdata.clear();
  v.win_len = 0;
  drop_staged(v);
  touched_[lane] = 0;
}

void GpuBackend_t::Stop(const TestcaseResult_t &Res) { cur().result = Res; }

void GpuBackend_t::SetLimit(const uint64_t Limit) {
  limit_ = Limit;
  if (ctx_) wtfgpu_set_limit(ctx_, Limit);
}

uint64_t GpuBackend_t::GetReg(const Registers_t Reg) {
  const int i = gpr_index(Reg);
  if (i >= 0) return cur().gpr[i];
  if (Reg == Registers_t::Cr2 || Reg == Registers_t::Cr3) {  // the lane's own (bochscpu_cpu_cr2/cr3)
    const int k = Reg == Registers_t::Cr2 ? 0 : 1;
    LaneView &v = cur();
    if (!(v.cr_known & (1 << k))) {
      std::lock_guard<std::mutex> g(engine_mu_);
      if (wtfgpu_lane_get_cr(ctx_, cur_, k ? 3 : 2, &v.cr[k]) != WTFGPU_OK) std::abort();
      v.cr_known |= uint8_t(1 << k);
    }
    return v.cr[k];
  }
  return 0;
}

uint64_t GpuBackend_t::SetReg(const Registers_t Reg, const uint64_t Value) {
  const int i = gpr_index(Reg);
  if (i >= 0) {
    cur().gpr[i] = Value;
    cur().regs_dirty = true;
  } else if (Reg == Registers_t::Cr2 || Reg == Registers_t::Cr3) {
    const int k = Reg == Registers_t::Cr2 ? 0 : 1;
    cur().cr[k] = Value;
    cur().cr_known |= uint8_t(1 << k);
    cur().cr_dirty |= uint8_t(1 << k);
  }
  return Value;
}

// bochscpu_backend.cc:874-885, per-lane seed
uint64_t GpuBackend_t::Rdrand() { return wtf_rdrand(cur().seed); }

// BochscpuRunStats_t::Print (bochscpu_backend.h:25-37) of the last testcase
// Run() ran, then the engine's own counters
void GpuBackend_t::PrintRunStats() {
  PrintTestcaseRunStats(last_run_, aggregate_.size());
  printf("  Breakpoint services: %llu in %llu rounds\n", (unsigned long long)stats_.breakpoint_hits,
         (unsigned long long)stats_.rounds);
  printf("       Kernel time ms: %.2f\n", stats_.kernel_ms);
}

// bochscpu_backend.cc:337-346
bool GpuBackend_t::SetBreakpoint(const Gva_t Gva, const BreakpointHandler_t Handler) {
  if (ModuleInstances *I = ModuleInstances::Registering()) {  // a module copy's Init (module_instances.h)
    I->AddHandler(Gva.U64(), Handler);
    if (I->RegisteringIndex() > 0) return breakpoints_.count(Gva.U64()) != 0;
  }
  if (breakpoints_.count(Gva.U64())) {
    printf("/!\\ There is already a breakpoint at %#llx\n", (unsigned long long)Gva.U64());
    return false;
  }
  breakpoints_.emplace(Gva.U64(), Handler);
  std::vector<uint64_t> v;
  for (auto &kv : breakpoints_) v.push_back(kv.first);
  return wtfgpu_set_breakpoints(ctx_, v.data(), (uint32_t)v.size()) == WTFGPU_OK;
}

bool GpuBackend_t::SetBreakpoint(const Gva_t Gva, const BreakpointHandler_t Handler,
                                 const BreakpointAction_t &Action) {
  if (!SetBreakpoint(Gva, Handler)) return false;
  if (ModuleInstances::Registering() && ModuleInstances::Registering()->RegisteringIndex() > 0) return true;
  const char *Env = getenv("WTFGPU_DEVICE_BP_ACTIONS");
  if (Action.Kind == BreakpointAction_t::Kind_t::Host || (Env && Env[0] == '0')) return true;
  wtfgpu_bp_action_t A;
  memset(&A, 0, sizeof(A));
  A.gva = Gva.U64();
  if (Action.Kind == BreakpointAction_t::Kind_t::SimulateReturn) {
    A.kind = WTFGPU_BPACT_RETURN;
    A.value = Action.Return;
    if (Action.StringReg >= 0) {
      const int g = gpr_index((Registers_t)Action.StringReg);
      if (g < 0) return false;
      A.gprs[0] = (uint64_t)g + 1;
      A.gprs[1] = Action.StringMax;
    }
  } else if (Action.Kind == BreakpointAction_t::Kind_t::Feed) {
    A.kind = WTFGPU_BPACT_FEED;
    A.value = Action.Return;
    A.gprs[0] = (uint64_t)gpr_index((Registers_t)Action.Gprs[0]);
    A.gprs[1] = (uint64_t)gpr_index((Registers_t)Action.Gprs[1]);
    feed_action_ = true;
  } else if (Action.Kind == BreakpointAction_t::Kind_t::StopOk) {
    A.kind = WTFGPU_BPACT_STOP_OK;
  } else if (Action.Kind == BreakpointAction_t::Kind_t::Rdrand) {
    A.kind = WTFGPU_BPACT_RDRAND;
    A.gprs[0] = (uint64_t)gpr_index((Registers_t)Action.Gprs[0]);
  } else if (Action.Kind == BreakpointAction_t::Kind_t::StopWithArgs) {
    if (!Action.ArgsResult || Action.Return > 6) return false;
    A.kind = WTFGPU_BPACT_STOP_ARGS;
    A.value = Action.Return;
    args_results_[Gva.U64()] = Action.ArgsResult;
  } else {
    A.kind = WTFGPU_BPACT_SET_GPRS;
    memcpy(A.gprs, Action.Gprs, sizeof(A.gprs));
  }
  bp_actions_.push_back(A);
  return wtfgpu_set_breakpoint_actions(ctx_, bp_actions_.data(), (uint32_t)bp_actions_.size()) == WTFGPU_OK;
}

bool GpuBackend_t::SetFeed(const uint8_t *Data, const uint64_t Size) {
  // the device serves the Feed action unless actions are off or the feed
  // does not fit a lane's feed region (wtfgpu_set_feed_lanes): then the
  // module's host handler must have its own copy
  if (!feed_action_ || Size > kFeedRegion) return false;
  LaneView &v = cur();
  v.has_feed = true;
  v.feed.assign(Data, Data + Size);
  return true;
}

// InsertAction_t on the device (wtfgpu_set_insert): every feed upload also
// inserts the lanes' testcases. Off with device actions off.
bool GpuBackend_t::DeclareInsert(const InsertAction_t &Action) {
  if (ModuleInstances::Registering() && ModuleInstances::Registering()->RegisteringIndex() > 0) return insert_action_;
  const char *Env = getenv("WTFGPU_DEVICE_BP_ACTIONS");
  if (Env && Env[0] == '0') return false;
  const int h = gpr_index(Action.HeadReg), p = gpr_index(Action.PtrReg), l = gpr_index(Action.LenReg);
  if (h < 0 || p < 0 || l < 0 || Action.LenArg > 64) return false;
  const wtfgpu_insert_t I = {(uint32_t)h, (uint32_t)p, (uint32_t)l, Action.LenArg};
  if (wtfgpu_set_insert(ctx_, &I) != WTFGPU_OK) return false;
  insert_action_ = true;
  return true;
}

// The testcase as the feed's one chunk (u32 size, bytes); the device applies
// the declared insert to it before the lane runs.
bool GpuBackend_t::SetInsert(const uint8_t *Data, const uint64_t Size) {
  if (!insert_action_ || Size + 4 > kFeedRegion) return false;
  LaneView &v = cur();
  v.has_feed = true;
  v.feed.resize(Size + 4);
  const uint32_t n = (uint32_t)Size;
  memcpy(v.feed.data(), &n, 4);
  if (Size) memcpy(v.feed.data() + 4, Data, Size);
  return true;
}

// One wtfgpu_set_feed call for lanes [0, n); lanes without SetFeed keep the
// host handler.
int GpuBackend_t::upload_feed(uint32_t n) {
  if (!(feed_action_ || insert_action_) || n == 0) return WTFGPU_OK;
  std::vector<uint64_t> off(n + 1);
  std::vector<uint8_t> has(n);
  uint64_t total = 0;
  for (uint32_t l = 0; l < n; l++) total += view(l).feed.size();
  std::vector<uint8_t> bytes;
  bytes.reserve(total);
  for (uint32_t l = 0; l < n; l++) {
    off[l] = bytes.size();
    has[l] = view(l).has_feed;
    bytes.insert(bytes.end(), view(l).feed.begin(), view(l).feed.end());
  }
  off[n] = bytes.size();
  return wtfgpu_set_feed(ctx_, 0, n, off.data(), has.data(), bytes.data(), bytes.size());
}

// Writes go to lane overlays, which the device dirties by itself.
bool GpuBackend_t::DirtyGpa(const Gpa_t) { return true; }

namespace {
constexpr size_t kArenaBlock = 16u << 20;  // 4096 staging slots per block
const uint8_t kZeroPage[Page::Size] = {};
}  // namespace

size_t GpuBackend_t::alloc_slots(size_t n, uint8_t **orig, uint8_t **data) const {
  // a thread inside a HostPool loop has its own arena (its index); any call
  // outside a loop takes the spare arena (index Threads()) under a lock, so a
  // second driver thread, whose loop ran serially because another thread held
  // the pool, never shares arena 0 with that loop's caller
  const bool in_loop = HostPool::InLoop();
  // shared with other allocations, exclusive with recycle_arenas: the slots
  // are counted as live (live_staged_) before a recycle can look
  std::shared_lock<std::shared_mutex> recycling(recycle_mu_);
  std::unique_lock<std::mutex> spare(spare_mu_, std::defer_lock);
  if (!in_loop) spare.lock();
  Arena &A = arenas_[in_loop ? HostPool::ThreadIndex() : arenas_.size() - 1];
  while (A.cur < A.blocks.size() && A.blocks[A.cur].cap - A.blocks[A.cur].used < n) A.cur++;
  if (A.cur == A.blocks.size()) {
    Block b;
    b.cap = std::max<size_t>(n, kArenaBlock / Page::Size);
    void *p = nullptr;
    int rc;
    {
      std::lock_guard<std::mutex> g(engine_mu_);
      rc = wtfgpu_host_alloc(ctx_, b.cap * Page::Size, &p);
    }
    if (rc != WTFGPU_OK) {
      printf("wtfgpu_host_alloc failed\n");
      std::abort();
    }
    b.orig = (uint8_t *)p;
    b.data.reset(new uint8_t[b.cap * Page::Size]);
    A.blocks.push_back(std::move(b));
  }
  Block &b = A.blocks[A.cur];
  *orig = b.orig + b.used * Page::Size;
  *data = b.data.get() + b.used * Page::Size;
  const size_t first = b.used;
  b.used += n;
  live_staged_ += n;  // reserved here, each one staged (stage) or released (release_slots)
  return first;
}

void GpuBackend_t::release_slots(size_t n) const { live_staged_ -= n; }

bool GpuBackend_t::parallel_service(const ModuleSlots *slots) const {
  return slots && slots->ThreadSafe() && HostPool::Get().Threads() > 1;
}

uint8_t *GpuBackend_t::stage(uint32_t lane, uint64_t gpfn, const uint8_t *orig, uint8_t *data) const {
  // orig / data: slots alloc_slots counted as live, or (orig only) a dump or
  // zero page with a fresh slot for data
  LaneView &v = view(lane);
  v.pages.push_back(Staged{gpfn, data, orig});
  for (LaneView::Logged &w : v.wlog)  // logged writes to this page move into it
    if (w.len && (w.gpa >> 12) == gpfn) {
      memcpy(data + (w.gpa & 0xfff), v.wdata.data() + w.off, w.len);
      w.len = 0;
    }
  return data;
}

// A handler's write to a page that is not staged is logged (gpa, bytes)
// instead of fetching the page: handlers mostly write buffers they never read
// back (the tlv packet, the hevd IOCTL buffer). Flush turns the log into
// device write records. Size stays within one page (Backend_t::VirtWrite).
bool GpuBackend_t::PhysWriteDirect(const Gpa_t Gpa, const uint8_t *Buffer, const uint64_t Size) {
  const uint32_t lane = cur_;
  if (Staged *p = find_staged(lane, Gpa.U64() >> 12)) {
    memcpy(p->data + (Gpa.U64() & 0xfff), Buffer, Size);
    return true;
  }
  LaneView &v = view(lane);
  if (v.win_len && Gpa.U64() < v.win_gpa + v.win_len && Gpa.U64() + Size > v.win_gpa) {  // keep the window current
    const uint64_t lo = std::max(Gpa.U64(), v.win_gpa), hi = std::min(Gpa.U64() + Size, v.win_gpa + v.win_len);
    memcpy(v.win + (lo - v.win_gpa), Buffer + (lo - Gpa.U64()), hi - lo);
  }
  if (!v.wlog.empty()) {  // coalesce with the previous write when it ends where this one starts
    LaneView::Logged &last = v.wlog.back();
    if (last.len && last.off + last.len == v.wdata.size() && last.gpa + last.len == Gpa.U64() &&
        ((last.gpa ^ Gpa.U64()) >> 12) == 0) {
      last.len += (uint32_t)Size;
      v.wdata.insert(v.wdata.end(), Buffer, Buffer + Size);
      return true;
    }
  }
  v.wlog.push_back(LaneView::Logged{Gpa.U64(), (uint32_t)Size, (uint32_t)v.wdata.size()});
  v.wdata.insert(v.wdata.end(), Buffer, Buffer + Size);
  return true;
}

// Reads of clean snapshot pages come straight from the dump (no staging copy);
// staged pages from their copy; overlay pages and pages with logged writes
// take the PhysTranslate path (fetch / prefetch, then staged).
bool GpuBackend_t::PhysReadDirect(const Gpa_t Gpa, uint8_t *Buffer, const uint64_t Size) const {
  const uint32_t lane = cur_;
  const uint64_t gpfn = Gpa.U64() >> 12;
  if (Staged *p = find_staged(lane, gpfn)) {
    memcpy(Buffer, p->data + (Gpa.U64() & 0xfff), Size);
    return true;
  }
  const LaneView &v = view(lane);
  if (v.win_len && Gpa.U64() >= v.win_gpa && Gpa.U64() + Size <= v.win_gpa + v.win_len) {
    memcpy(Buffer, v.win + (Gpa.U64() - v.win_gpa), Size);
    return true;
  }
  if (!v.dirty_known || in_overlay(v, gpfn)) return false;
  for (const LaneView::Logged &w : v.wlog)
    if (w.len && (w.gpa >> 12) == gpfn) return false;
  const uint8_t *p = dump_.GetPhysicalPage(gpfn << 12);
  memcpy(Buffer, (p ? p : kZeroPage) + (Gpa.U64() & 0xfff), Size);
  return true;
}

uint8_t *GpuBackend_t::stage_copy(uint32_t lane, uint64_t gpfn, const uint8_t *orig) const {
  uint8_t *o, *d;
  alloc_slots(1, &o, &d);
  memcpy(d, orig, Page::Size);
  return stage(lane, gpfn, orig, d);
}

void GpuBackend_t::drop_staged(LaneView &v) const {
  if (v.pages.empty()) return;
  live_staged_ -= v.pages.size();
  v.pages.clear();
  if (!HostPool::InLoop()) recycle_arenas();
}

// Every staged page consumed: the arenas start over (outside HostPool loops
// only; callers of parallel drop_staged call it after their loop).
void GpuBackend_t::recycle_arenas() const {
  if (live_staged_ != 0 || HostPool::InLoop()) return;
  std::unique_lock<std::shared_mutex> recycling(recycle_mu_);
  if (live_staged_ != 0) return;  // an allocation came in between
  std::lock_guard<std::mutex> spare(spare_mu_);
  for (Arena &A : arenas_) {
    for (Block &b : A.blocks) b.used = 0;
    A.cur = 0;
  }
}

GpuBackend_t::Staged *GpuBackend_t::find_staged(uint32_t lane, uint64_t gpfn) const {
  for (Staged &p : view(lane).pages)
    if (p.gpfn == gpfn) return &p;
  return nullptr;
}

bool GpuBackend_t::in_overlay(const LaneView &v, uint64_t gpfn) const {
  return std::find(v.dirty.begin(), v.dirty.end(), (uint32_t)gpfn) != v.dirty.end();
}

// The lane's view of a physical page, on the host: staged copy, else a fetch of
// the lane's overlay page, else the dump page (or zeros).
uint8_t *GpuBackend_t::lane_page(uint32_t lane, uint64_t gpfn) const {
  if (Staged *p = find_staged(lane, gpfn)) return p->data;
  LaneView &v = view(lane);
  if (!v.dirty_known) {
    std::vector<uint32_t> buf(overlay_pages_ + 1);
    std::lock_guard<std::mutex> g(engine_mu_);
    wtfgpu_read_dirty_list(ctx_, &lane, 1, buf.data());
    v.dirty.assign(buf.begin() + 1, buf.begin() + 1 + std::min<uint32_t>(buf[0], overlay_pages_));
    v.dirty_known = true;
  }
  if (in_overlay(v, gpfn)) {
    const auto t0 = Clock::now();
    uint8_t *o, *d;
    alloc_slots(1, &o, &d);
    const uint64_t gpa = gpfn << 12;
    std::lock_guard<std::mutex> g(engine_mu_);
    wtfgpu_gather_pages(ctx_, &lane, &gpa, 1, o);
    memcpy(d, o, Page::Size);
    stats_.page_fetches++;
    stats_.fetch_ms += ms_since(t0);
    fetch_by_bp_[servicing_bp_]++;
    learn(gpfn);
    return stage(lane, gpfn, o, d);
  }
  if (scouting_) learn(gpfn);  // serial: no other thread reads or writes the tables
  const uint8_t *p = dump_.GetPhysicalPage(gpfn << 12);
  return stage_copy(lane, gpfn, p ? p : kZeroPage);
}

// Learned prefetch: the breakpoint being serviced touched frame `gpfn`
// (caller holds engine_mu_ or runs serially).
void GpuBackend_t::learn(uint64_t gpfn) const {
  if (servicing_bp_ == ~0ull) return;
  if (gpfn == servicing_sp_) {
    bp_stack_.insert(servicing_bp_);
    return;
  }
  auto &l = bp_pages_[servicing_bp_];
  if (l.size() < 8 && std::find(l.begin(), l.end(), gpfn) == l.end()) l.push_back(gpfn);
}

const uint8_t *GpuBackend_t::lane_page_ro(uint32_t lane, uint64_t gpfn) const {
  if (Staged *p = find_staged(lane, gpfn)) return p->data;
  const LaneView &v = view(lane);
  if (!v.dirty_known || in_overlay(v, gpfn)) return lane_page(lane, gpfn);
  const uint8_t *p = dump_.GetPhysicalPage(gpfn << 12);
  return p ? p : kZeroPage;
}

// bochscpu_mem_virt_translate semantics (present bits only), on the lane view
// Walk memo (per host thread, direct mapped): a walk that read only snapshot
// page-table pages (none staged or in the lane's overlay) holds for every lane
// whose view does not hold those table frames either, so it is reused after a
// per-lane check of at most four frames instead of a four-level walk.
namespace {
struct WalkMemo {
  uint64_t vpn = ~0ull, base = 0, mask = 0;
  uint64_t tables[4] = {};
  uint32_t ntables = 0;
};
thread_local WalkMemo t_walk_memo[64];
}  // namespace

bool GpuBackend_t::VirtTranslate(const Gva_t Gva, Gpa_t &Gpa, const MemoryValidate_t) const {
  const uint64_t va = Gva.U64(), vpn = va >> 12;
  const LaneView &v = view(cur_);
  WalkMemo &m = t_walk_memo[vpn & 63];
  if (m.vpn == vpn && v.dirty_known && (!(v.cr_known & 2) || v.cr[1] == initial_.Cr3)) {
    bool clean = true;
    for (uint32_t k = 0; k < m.ntables && clean; k++)
      clean = !in_overlay(v, m.tables[k]) && !find_staged(cur_, m.tables[k]);
    if (clean) {
      Gpa = Gpa_t(m.base | (va & m.mask));
      return true;
    }
  }
  uint64_t table = initial_.Cr3 & 0x000ffffffffff000ull;
  WalkMemo w;
  bool from_dump = v.dirty_known;
  if ((v.cr_known & 2) && v.cr[1] != initial_.Cr3) {  // a handler moved the lane's cr3
    table = v.cr[1] & 0x000ffffffffff000ull;
    from_dump = false;  // not memoised: the memo holds walks from the snapshot's cr3
  }
  for (int level = 3; level >= 0; level--) {
    const uint64_t tf = table >> 12;
    w.tables[w.ntables++] = tf;
    from_dump = from_dump && !in_overlay(v, tf) && !find_staged(cur_, tf);
    const uint8_t *pg = lane_page_ro(cur_, tf);
    uint64_t e;
    memcpy(&e, pg + ((va >> (12 + 9 * level)) & 0x1ff) * 8, 8);
    if (!(e & 1)) return false;
    const uint64_t frame = e & 0x000ffffffffff000ull;
    if ((level == 2 || level == 1) && (e & 0x80)) {
      w.mask = level == 2 ? 0x3fffffffull : 0x1fffffull;
      w.base = frame & ~w.mask;
      break;
    }
    if (level == 0) {
      w.mask = 0xfff;
      w.base = frame;
    }
    table = frame;
  }
  Gpa = Gpa_t(w.base | (va & w.mask));
  if (from_dump) {
    w.vpn = vpn;
    m = w;
  }
  return true;
}

// A host pointer into the lane's staged copy of the page: writes through it are
// diffed against the original at flush time and applied to the lane overlay.
uint8_t *GpuBackend_t::PhysTranslate(const Gpa_t Gpa) const {
  return lane_page(cur_, Gpa.U64() >> 12) + (Gpa.U64() & 0xfff);
}

// bochscpu_backend.cc:902-999: the first page of the range that does not
// translate gets a #PF(Write|User) injected when the handler returns; the guest
// pages it in and re-executes the hooked instruction (its breakpoint fires again).
bool GpuBackend_t::PageFaultsMemoryIfNeeded(const Gva_t Gva, const uint64_t Size) {
  for (uint64_t a = Gva.U64() & ~0xfffull; a < Gva.U64() + Size; a += Page::Size) {
    Gpa_t G;
    if (!VirtTranslate(Gva_t(a), G, MemoryValidate_t::ValidateRead)) {
      cur().inject = a;
      return true;
    }
  }
  return false;
}

const std::unordered_set<Gva_t> &GpuBackend_t::LastNewCoverage() const { return last_new_coverage_; }

// bochscpu_backend.cc:1005-1016
bool GpuBackend_t::RevokeLastNewCoverage() {
  for (const Gva_t &g : last_new_coverage_) aggregate_.erase(g.U64());
  last_new_coverage_.clear();
  return true;
}

// Staged registers and memory of `lanes` -> device. Pages are diffed against
// their original content in parallel; each changed byte range becomes one
// write record (copy-on-write + dirty on the device).
int GpuBackend_t::flush_lanes(const std::vector<uint32_t> &lanes) {
  const auto tp = Clock::now();
  const size_t nl = lanes.size();
  const bool par = nl >= 1024;
  // per lane: registers to upload, staged pages, logged write records / bytes
  // (counted on all host threads, then prefix sums)
  std::vector<uint64_t> rcnt(nl + 1, 0), pcnt(nl + 1, 0), roff(nl + 1, 0), boff(nl + 1, 0);
  std::atomic<bool> any_cr{false};
  HostPool::Get().For(nl, 256, [&](size_t i) {
    const LaneView &v = view(lanes[i]);
    rcnt[i + 1] = v.regs_dirty ? 1 : 0;
    pcnt[i + 1] = v.pages.size();
    uint64_t r = 0, b = 0;
    for (const LaneView::Logged &w : v.wlog)
      if (w.len) {
        r++;
        b += w.len;
      }
    roff[i + 1] = r;
    boff[i + 1] = b;
    if (v.cr_dirty) any_cr.store(true, std::memory_order_relaxed);
  }, par);
  for (size_t i = 0; i < nl; i++) {
    rcnt[i + 1] += rcnt[i];
    pcnt[i + 1] += pcnt[i];
    roff[i + 1] += roff[i];
    boff[i + 1] += boff[i];
  }
  if (any_cr)
    for (uint32_t l : lanes) {
      LaneView &v = view(l);
      for (int k = 0; k < 2; k++)
        if (v.cr_dirty & (1 << k)) {
          std::lock_guard<std::mutex> g(engine_mu_);
          if (wtfgpu_lane_set_cr(ctx_, l, k ? 3 : 2, v.cr[k]) != WTFGPU_OK) return WTFGPU_ERR_INVALID;
        }
      v.cr_dirty = 0;
    }
  std::vector<uint32_t> rl(rcnt[nl]);
  std::vector<uint64_t> regs(rcnt[nl] * 18);
  // staged pages: diffed against their original content, only the changed span is written
  struct Cand {
    uint32_t lane;
    const Staged *p;
    uint32_t lo, hi;
  };
  std::vector<Cand> cand(pcnt[nl]);
  HostPool::Get().For(nl, 256, [&](size_t i) {
    const uint32_t l = lanes[i];
    LaneView &v = view(l);
    if (v.regs_dirty) {
      rl[rcnt[i]] = l;
      memcpy(&regs[rcnt[i] * 18], v.gpr, 18 * 8);
      v.regs_dirty = false;
    }
    uint64_t k = pcnt[i];
    for (const Staged &p : v.pages) cand[k++] = Cand{l, &p, 0, 0};
  }, par);
  HostPool::Get().For(cand.size(), 64, [&](size_t i) {
    const uint8_t *d = cand[i].p->data, *o = cand[i].p->orig;
    if (!memcmp(d, o, Page::Size)) return;
    size_t lo = 0, hi = Page::Size;
    while (lo + 8 <= hi && !memcmp(d + lo, o + lo, 8)) lo += 8;
    while (lo < hi && d[lo] == o[lo]) lo++;
    while (hi >= lo + 8 && !memcmp(d + hi - 8, o + hi - 8, 8)) hi -= 8;
    while (hi > lo && d[hi - 1] == o[hi - 1]) hi--;
    cand[i].lo = (uint32_t)lo;
    cand[i].hi = (uint32_t)hi;
  });
  // the write records and their bytes, laid out per lane and filled on all
  // host threads into a pinned buffer: one DMA to the device
  uint64_t cbytes = 0, crecs = 0;
  for (const Cand &c : cand)
    if (c.lo != c.hi) {
      crecs++;
      cbytes += c.hi - c.lo;
    }
  std::vector<wtfgpu_write_t> writes(roff[nl] + crecs);
  const uint64_t total = boff[nl] + cbytes;
  if (total > wpin_cap_) {
    if (wpin_) wtfgpu_host_free(ctx_, wpin_);
    wpin_ = nullptr;
    wpin_cap_ = std::max<uint64_t>(total * 2, 1 << 20);
    void *p = nullptr;
    if (wtfgpu_host_alloc(ctx_, wpin_cap_, &p)) return WTFGPU_ERR_OOM;
    wpin_ = (uint8_t *)p;
  }
  HostPool::Get().For(nl, 256, [&](size_t i) {
    const uint32_t l = lanes[i];
    LaneView &v = view(l);
    uint64_t r = roff[i], b = boff[i];
    for (const LaneView::Logged &w : v.wlog) {
      if (!w.len) continue;
      writes[r++] = wtfgpu_write_t{l, w.len, w.gpa, b};
      memcpy(wpin_ + b, v.wdata.data() + w.off, w.len);
      b += w.len;
      v.dirty_known = false;
    }
    v.wlog.clear();
    v.wdata.clear();
  }, par);
  {
    uint64_t r = roff[nl], b = boff[nl];
    for (const Cand &c : cand) {
      if (c.lo == c.hi) continue;
      wtfgpu_write_t w{};
      w.lane = c.lane;
      w.len = c.hi - c.lo;
      w.gva = (c.p->gpfn << 12) | c.lo;
      w.data_off = b;
      memcpy(wpin_ + b, c.p->data + c.lo, w.len);
      b += w.len;
      writes[r++] = w;
      view(c.lane).dirty_known = false;  // the device overlay changed
    }
  }
  stats_.staged_pages += cand.size();
  if (!cand.empty())
    for (uint32_t l : lanes) drop_staged(view(l));
  int rc = WTFGPU_OK;
  const auto tr = Clock::now();
  stats_.up_prep_ms += std::chrono::duration<double, std::milli>(tr - tp).count();
  if (!rl.empty()) rc = wtfgpu_write_gprs_list(ctx_, rl.data(), (uint32_t)rl.size(), regs.data());
  const auto ta = Clock::now();
  stats_.up_regs_ms += std::chrono::duration<double, std::milli>(ta - tr).count();
  if (!rc && !writes.empty())
    rc = wtfgpu_apply_phys_writes(ctx_, writes.data(), (uint32_t)writes.size(), wpin_, total, nullptr);
  stats_.up_apply_ms += ms_since(ta);
  return rc;
}

// One round's exits: each pending lane that is not done is classified (a
// result, or a breakpoint hit for the host, or still running). A device Feed
// action that could not write its chunk (WTFGPU_EXIT_FEED_FAULT) is the
// module handler's failed VirtWriteDirty (fuzzer_tlv_server.cc:130-158): a
// handler fault, the testcase an engine error (U43).
bool GpuBackend_t::classify(const std::vector<uint32_t> &pending, uint32_t first, const wtfgpu_exit_t *ex,
                            std::vector<uint8_t> &done, std::vector<LaneResult> *out, std::vector<uint32_t> &hits,
                            const uint64_t *stop_args) {
  std::vector<uint8_t> hit(pending.size(), 0);
  HostPool::Get().For(pending.size(), 1024, [&](size_t pi) {
    const uint32_t l = pending[pi];
    if (done[l - first]) return;
    const wtfgpu_exit_t &e = ex[l - first];
    // a view the host has not touched since its reset holds no result: the
    // common exits (Stop(Ok), still running, a breakpoint) leave it so
    LaneView &v = views_[l];
    const auto mark = [&]() -> LaneView & {
      touched_[l] = 1;
      return v;
    };
    switch (e.status) {
      case WTFGPU_EXIT_BREAKPOINT: hit[pi] = 1; return;
      case WTFGPU_RUNNING: return;  // sliced: still running when the slice ended
      case WTFGPU_EXIT_TIMEOUT: mark().result = Timedout_t(); break;  // bochscpu_backend.cc:458-469
      case WTFGPU_EXIT_INT3:                                           // :595-619
      case WTFGPU_EXIT_HLT: mark().result = Crash_t(); break;          // :690-697
      case WTFGPU_EXIT_CR3: mark().result = Cr3Change_t(); break;      // :628-657
      case WTFGPU_EXIT_FAULT: mark().result = FaultToResult(e.vector, e.error, e.rip, e.addr, e.opcode); break;
      case WTFGPU_EXIT_STOPPED: break;
      case WTFGPU_EXIT_STOP_OK:  // device Feed action: Stop(Ok_t()) (an untouched view reads as Ok already)
        if (touched_[l]) v.result = Ok_t();
        break;
      case WTFGPU_EXIT_STOP_ARGS: hit[pi] = 2; return;                  // named below from the kept arguments
      case WTFGPU_EXIT_FEED_FAULT: mark().handler_fault = true; break;  // U43: fill_results makes it an engine error
      default:
        // unimplemented opcode / overlay full / a device Feed write that
        // failed: the engine cannot finish the testcase. Not a target bug:
        // flagged as an engine error, with an unnamed Crash_t (which no
        // master saves, server.h:861-877) as its result
        if (out) (*out)[l].error = true;
        if (!v.result) mark().result = Crash_t();
        if (e.status == WTFGPU_EXIT_UNIMPLEMENTED) {
          stats_.err_unimpl++;
          stats_.unimpl_ops.add(e.opcode);
          stats_.last_unimpl_op = e.opcode;
          stats_.last_unimpl_rip = e.rip;
        } else if (e.status == WTFGPU_EXIT_OVERLAY_FULL) {
          stats_.err_overlay++;
        } else {
          stats_.err_other++;
        }
        break;
    }
    done[l - first] = 1;
  }, pending.size() >= 2048);
  std::vector<uint32_t> named;
  for (size_t pi = 0; pi < pending.size(); pi++) {
    if (hit[pi] == 1) hits.push_back(pending[pi]);
    if (hit[pi] == 2) named.push_back(pending[pi]);
  }
  if (named.empty()) return true;
  // device StopWithArgs actions: the handler's Stop(Result(GetArg(0..5)))
  std::vector<uint64_t> args(named.size() * 6);
  bool ok = true;
  if (stop_args) {
    HostPool::Get().For(named.size(), 2048, [&](size_t k) {
      memcpy(&args[k * 6], stop_args + (uint64_t)(named[k] - first) * 6, 48);
    }, named.size() >= 8192);
  } else {
    ok = wtfgpu_read_stop_args(ctx_, named.data(), (uint32_t)named.size(), args.data()) == WTFGPU_OK;
  }
  std::atomic<uint64_t> bad{0};
  HostPool::Get().For(named.size(), 512, [&](size_t k) {
    const uint32_t l = named[k];
    LaneView &v = view(l);
    const auto it = args_results_.find(ex[l - first].rip);
    if (ok && it != args_results_.end()) {
      v.result = it->second(&args[k * 6]);
    } else {  // cannot happen unless the engine misbehaves: an engine error, not a target bug
      if (out) (*out)[l].error = true;
      if (!v.result) v.result = Crash_t();
      bad++;
    }
    done[l - first] = 1;
  }, named.size() >= 2048);
  stats_.err_other += bad;
  return true;
}

// Final state of every finished lane (`ex` holds the last round's exits of
// every lane: a lane is final once it is done).
bool GpuBackend_t::fill_results(const std::vector<uint32_t> &lanes, uint32_t first,
                                const wtfgpu_exit_t *ex, const std::vector<uint8_t> &done,
                                std::vector<LaneResult> *out, std::vector<uint32_t> *finished) {
  const auto tg = Clock::now();
  std::vector<uint32_t> fin;
  for (uint32_t l : lanes)
    if (done[l - first]) fin.push_back(l);
  if (finished) finished->insert(finished->end(), fin.begin(), fin.end());
  if (!out) return true;
  std::vector<uint64_t> regs;
  // run stats of [lo, hi) (run mode): byte, dirty-page and edge counters
  uint32_t lo = 0, hi = 0;
  std::vector<uint64_t> nb;
  std::vector<uint32_t> dc, ec;
  if (want_gprs_) {  // run mode prints them; the fuzz loop never reads them
    regs.resize(fin.size() * 18);
    if (!fin.empty() && wtfgpu_read_gprs_list(ctx_, fin.data(), (uint32_t)fin.size(), regs.data())) return false;
    if (!fin.empty()) {
      lo = *std::min_element(fin.begin(), fin.end());
      hi = *std::max_element(fin.begin(), fin.end()) + 1;
      nb.resize(hi - lo);
      dc.resize(hi - lo);
      ec.resize(2 * (hi - lo));
      if (wtfgpu_read_bytes(ctx_, lo, hi - lo, nb.data()) || wtfgpu_read_dirty_counts(ctx_, lo, hi - lo, dc.data()) ||
          wtfgpu_read_edge_counts(ctx_, lo, hi - lo, ec.data()))
        return false;
    }
  }
  HostPool::Get().For(fin.size(), 1024, [&](size_t i) {
    LaneResult &r = (*out)[fin[i]];
    const LaneView &v = views_[fin[i]];  // untouched since its reset: no result, no fault
    const bool t = touched_[fin[i]] != 0;
    r.result = t && v.result ? std::move(*v.result) : TestcaseResult_t(Ok_t());  // the view is reset at refill
    if (t && v.handler_fault) {  // U43: an engine error, never a named crash
      r.result = Crash_t();
      r.error = true;
      r.handler_fault = true;
      stats_.err_handler++;
    }
    if (want_gprs_) {
      memcpy(r.gprs, &regs[i * 18], 18 * 8);
      r.rip = r.gprs[16];
      const uint32_t k = fin[i] - lo;
      r.bytes = nb[k];
      r.dirty = std::min(dc[k], overlay_pages_);
      r.edges = ec[2 * k];
      r.edges_new = ec[2 * k + 1];
    } else {
      r.rip = ex[fin[i] - first].rip;
    }
    r.icount = ex[fin[i] - first].icount;
    r.exit_status = ex[fin[i] - first].status;
  }, fin.size() >= 2048);
  stats_.regs_ms += ms_since(tg);
  return true;
}

// Lanes InsertTestcase stopped never run: marked STOPPED on the device, so
// the next classification gives them their result.
bool GpuBackend_t::stop_prestopped(const std::vector<uint32_t> &lanes) {
  std::vector<uint8_t> has(lanes.size());
  HostPool::Get().For(lanes.size(), 1024, [&](size_t i) { has[i] = touched_[lanes[i]] && views_[lanes[i]].result.has_value(); },
                      lanes.size() >= 4096);
  std::vector<uint32_t> pre;
  for (size_t i = 0; i < lanes.size(); i++)
    if (has[i]) pre.push_back(lanes[i]);
  return pre.empty() || wtfgpu_stop(ctx_, pre.data(), (uint32_t)pre.size(), WTFGPU_EXIT_STOPPED) == WTFGPU_OK;
}

// The run loop over `lanes` (ascending): launch, classify exits, service
// breakpoint hits on the host, resume; until every lane has a result.
bool GpuBackend_t::run_lanes(const std::vector<uint32_t> &lanes, std::vector<LaneResult> *out, ModuleSlots *slots,
                             bool per_lane_state) {
  if (lanes.empty()) return true;
  const uint32_t first = lanes.front() & ~63u, count = lanes.back() + 1 - first;
  std::vector<wtfgpu_exit_t> ex(count);
  std::vector<uint8_t> done(count, 0);
  std::vector<uint32_t> pending = lanes;
  if (!stop_prestopped(lanes)) return false;
  for (;;) {
    wtfgpu_run_stats_t rs{};
    const auto tk = Clock::now();
    if (wtfgpu_run(ctx_, first, count, ~0ull, &rs)) return false;
    const auto te = Clock::now();
    stats_.run_ms += std::chrono::duration<double, std::milli>(te - tk).count();
    account_run(rs);
    if (wtfgpu_read_exits(ctx_, first, count, ex.data())) return false;
    std::vector<uint32_t> hits;
    if (!classify(pending, first, ex.data(), done, out, hits)) return false;
    stats_.exits_ms += ms_since(te);
    if (hits.empty()) break;
    if (!service_hits(hits, first, done, slots, per_lane_state)) return false;
    pending.clear();
    for (uint32_t l : hits)
      if (!done[l - first]) pending.push_back(l);
  }
  return fill_results(lanes, first, ex.data(), done, out, nullptr);
}

void GpuBackend_t::account_run(const wtfgpu_run_stats_t &rs) {
  stats_.kernel_launches += rs.kernel_launches;
  stats_.kernel_ms += rs.kernel_ms;
  stats_.retired += rs.lane_retired;
  stats_.group_steps += rs.group_steps;
  stats_.rounds++;
}

// Services one round's breakpoint hits on the host (BeforeExecutionHook,
// bochscpu_backend.cc:476-548): bulk reads, prefetch, handlers (on all host
// threads when the module's state is thread_local), flush, then each lane is
// resumed or stopped (done[l - first] = 1).
bool GpuBackend_t::service_hits(const std::vector<uint32_t> &hits, uint32_t first, std::vector<uint8_t> &done,
                                ModuleSlots *slots, bool per_lane_state) {
  const auto t0 = Clock::now();
  {
    // ---- service the round's breakpoint hits
    std::vector<uint64_t> regs(hits.size() * 18);
    if (wtfgpu_read_gprs_list(ctx_, hits.data(), (uint32_t)hits.size(), regs.data())) return false;
    // the lanes' Rdrand chains (a device Rdrand action may have advanced them)
    std::vector<uint64_t> seeds(hits.size());
    if (wtfgpu_lane_seeds(ctx_, hits.data(), (uint32_t)hits.size(), seeds.data(), 0)) return false;
    const uint32_t stride = overlay_pages_ + 1;
    std::vector<uint32_t> dl(hits.size() * stride);
    if (wtfgpu_read_dirty_list(ctx_, hits.data(), (uint32_t)hits.size(), dl.data())) return false;
    const auto t1 = Clock::now();
    stats_.bulk_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
    // prefetch, in one bulk gather, the overlay frames the handlers will touch,
    // learned from the on-demand fetches of earlier hits of the same
    // breakpoint: its stack page (return address / arguments, bp_stack_) and
    // fixed frames (e.g. the tlv packet buffer, bp_pages_)
    std::vector<uint64_t> sp_gpfn(hits.size(), ~0ull), sp_gpa(hits.size(), ~0ull);
    // lane views of the hits (independent per lane: all host threads)
    HostPool::Get().For(hits.size(), 256, [&](size_t i) {
      LaneView &v = view(hits[i]);
      memcpy(v.gpr, &regs[i * 18], 18 * 8);
      v.seed = seeds[i];
      v.regs_dirty = false;
      v.cr_known = 0;  // an exception delivery or a cr write may have changed them
      v.win_len = 0;
      drop_staged(v);
      const uint32_t cnt = std::min(dl[i * stride], overlay_pages_);
      v.dirty.assign(dl.begin() + i * stride + 1, dl.begin() + i * stride + 1 + cnt);
      v.dirty_known = true;
      // the stack page is needed to learn (a breakpoint's first hit) or to
      // prefetch for breakpoints whose handler reads the stack
      const uint64_t rip = v.gpr[16];
      if (!bp_seen_.count(rip) || bp_stack_.count(rip)) {
        cur_ = hits[i];
        Gpa_t sp;
        if (VirtTranslate(Gva_t(v.gpr[WTFGPU_RSP]), sp, MemoryValidate_t::ValidateRead)) {
          sp_gpa[i] = sp.U64();
          sp_gpfn[i] = sp.U64() >> 12;
        }
      }
    });
    recycle_arenas();  // drop_staged ran inside the loop
    // the handlers: lane by lane, or on all host threads when the module keeps
    // its per-testcase state thread_local (each thread services its own lanes
    // with g_Backend = this and its own swapped-in module state). The order of
    // lanes does not matter: every lane has its own view and module state.
    std::vector<uint8_t> action(hits.size());  // 0 stop, 1 resume, 2 resume + skip the breakpoint
    auto service = [&](size_t h) {
      const uint32_t l = hits[h];
      LaneView &v = view(l);
      cur_ = l;
      const uint64_t rip0 = v.gpr[16];
      servicing_sp_ = sp_gpfn[h];
      BreakpointHandler_t handler = nullptr;
      if (slots && slots->Instances()) {
        handler = slots->Instances()->HandlerOf(l, rip0);  // lane l's module copy
      } else {
        const auto it = breakpoints_.find(rip0);
        if (it != breakpoints_.end()) handler = it->second;
      }
      if (per_lane_state && slots) slots->SwapIn(l);
      servicing_bp_ = rip0;
      v.inject = ~0ull;
      try {
        if (handler) handler(this);  // BeforeExecutionHook (bochscpu_backend.cc:545-547)
      } catch (const HandlerFault_t &) {  // the reference node stops here (backend.cc:39-42): this lane does
        v.handler_fault = true;
        v.result = Crash_t();
      }
      servicing_bp_ = ~0ull;
      if (per_lane_state && slots) slots->SwapOut(l);
      action[h] = v.result ? 0 : (v.gpr[16] == rip0 ? 2 : 1);  // U10: a moved rip cancels the hooked instruction
    };
    Backend_t *saved = g_Backend;
    g_Backend = this;
    // scouts: the first hit of a breakpoint never serviced before runs alone
    // first, so its on-demand page fetches teach the prefetcher (below) what
    // the other lanes' handlers will touch
    std::vector<uint8_t> scouted(hits.size(), 0);
    for (size_t i = 0; i < hits.size(); i++) {
      if (!bp_seen_.insert(view(hits[i]).gpr[16]).second) continue;
      scouting_ = true;
      service(i);
      scouting_ = false;
      scouted[i] = 1;
    }
    // prefetch, in one bulk gather, the overlay frames the handlers will touch,
    // learned from the on-demand fetches of earlier hits of the same
    // breakpoint: its stack page (return address / arguments, bp_stack_) and
    // fixed frames (e.g. the tlv packet buffer, bp_pages_)
    // The stack is fetched as a kWin-byte window at [rsp] (return address and
    // stack arguments) when that window stays inside the page; handler reads
    // outside it fall back to the page path.
    std::vector<uint32_t> pf_lanes, win_lanes;
    std::vector<uint64_t> pf_gpas, win_gpas;
    std::vector<uint8_t> use_win(hits.size(), 0);
    HostPool::Get().For(hits.size(), 256, [&](size_t i) {
      if (scouted[i] || sp_gpfn[i] == ~0ull) return;
      const LaneView &v = view(hits[i]);
      if (bp_stack_.count(v.gpr[16]) && in_overlay(v, sp_gpfn[i]))
        use_win[i] = (sp_gpa[i] & 0xfff) + LaneView::kWin <= Page::Size ? 1 : 2;  // 2: whole page
    });
    for (size_t i = 0; i < hits.size(); i++) {
      if (scouted[i]) continue;
      const LaneView &v = view(hits[i]);
      auto want = [&](uint64_t gpfn) {
        if (!in_overlay(v, gpfn)) return;
        for (size_t k = pf_gpas.size(); k-- > 0 && pf_lanes[k] == hits[i];)
          if (pf_gpas[k] == gpfn << 12) return;
        pf_lanes.push_back(hits[i]);
        pf_gpas.push_back(gpfn << 12);
      };
      if (use_win[i] == 1) {
        win_lanes.push_back(hits[i]);
        win_gpas.push_back(sp_gpa[i]);
      } else if (use_win[i] == 2) {
        want(sp_gpfn[i]);
      }
      if (!bp_pages_.empty()) {
        auto lp = bp_pages_.find(v.gpr[16]);
        if (lp != bp_pages_.end())
          for (uint64_t g : lp->second) want(g);
      }
    }
    if (!win_lanes.empty()) {
      const size_t nw = win_lanes.size();
      std::vector<uint8_t> buf(nw * LaneView::kWin);
      if (wtfgpu_gather_bytes(ctx_, win_lanes.data(), win_gpas.data(), (uint32_t)nw, LaneView::kWin, buf.data()))
        return false;
      HostPool::Get().For(nw, 256, [&](size_t i) {
        LaneView &v = view(win_lanes[i]);
        v.win_gpa = win_gpas[i];
        v.win_len = LaneView::kWin;
        memcpy(v.win, buf.data() + i * LaneView::kWin, LaneView::kWin);
      });
      stats_.stack_windows += nw;
    }
    if (!pf_lanes.empty()) {
      const size_t np = pf_lanes.size();
      uint8_t *o, *d;
      alloc_slots(np, &o, &d);
      if (wtfgpu_gather_pages(ctx_, pf_lanes.data(), pf_gpas.data(), (uint32_t)np, o)) {
        release_slots(np);
        return false;
      }
      HostPool::Get().For(np, 256, [&](size_t i) { memcpy(d + i * Page::Size, o + i * Page::Size, Page::Size); });
      for (size_t i = 0; i < np; i++)
        stage(pf_lanes[i], pf_gpas[i] >> 12, o + i * Page::Size, d + i * Page::Size);
      stats_.prefetched_pages += np;
    }
    const auto t2 = Clock::now();
    stats_.prefetch_ms += std::chrono::duration<double, std::milli>(t2 - t1).count();
    if (per_lane_state && parallel_service(slots)) {
      HostPool::Get().For(hits.size(), 64, [&](size_t h) {
        g_Backend = this;
        if (!scouted[h]) service(h);
      });
    } else {
      for (size_t h = 0; h < hits.size(); h++)
        if (!scouted[h]) service(h);
    }
    g_Backend = saved;
    stats_.breakpoint_hits += hits.size();
    const auto t3 = Clock::now();
    stats_.handler_ms += std::chrono::duration<double, std::milli>(t3 - t2).count();
    if (flush_lanes(hits)) return false;
    for (size_t i = 0; i < hits.size(); i++) seeds[i] = view(hits[i]).seed;
    if (wtfgpu_lane_seeds(ctx_, hits.data(), (uint32_t)hits.size(), seeds.data(), 1)) return false;
    {  // PageFaultsMemoryIfNeeded requests: #PF through the guest IDT, resume at the handler
      std::vector<uint32_t> il;
      std::vector<uint64_t> ia;
      std::vector<size_t> ih;
      for (size_t h = 0; h < hits.size(); h++)
        if (action[h] != 0 && view(hits[h]).inject != ~0ull) {
          il.push_back(hits[h]);
          ia.push_back(view(hits[h]).inject);
          ih.push_back(h);
        }
      if (!il.empty()) {
        std::vector<int32_t> ok(il.size());
        if (wtfgpu_inject_fault(ctx_, il.data(), (uint32_t)il.size(), WTFGPU_VEC_PF, ErrorWrite | ErrorUser, ia.data(),
                                ok.data()))
          return false;
        for (size_t k = 0; k < il.size(); k++) {
          if (ok[k]) {
            action[ih[k]] = 1;  // resume at the handler, no breakpoint skip
          } else {
            view(il[k]).result = Crash_t();  // no IDT to take it: the triple fault bochs stops on
            action[ih[k]] = 0;
          }
        }
      }
    }
    std::vector<uint32_t> resume, stop;
    std::vector<uint8_t> skip;
    for (size_t h = 0; h < hits.size(); h++) {
      if (action[h] == 0) {
        stop.push_back(hits[h]);
        done[hits[h] - first] = 1;
      } else {
        resume.push_back(hits[h]);
        skip.push_back(action[h] == 2);
      }
    }
    if (!stop.empty() && wtfgpu_stop(ctx_, stop.data(), (uint32_t)stop.size(), WTFGPU_EXIT_STOPPED)) return false;
    if (!resume.empty() && wtfgpu_resume(ctx_, resume.data(), (uint32_t)resume.size(), skip.data())) return false;
    stats_.flush_ms += ms_since(t3);
    stats_.service_ms += ms_since(t0);
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
      if (n == 1)
        for (uint64_t rip : per[l]) last_new_coverage_.insert(Gva_t(rip));
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
  commit_fresh(fresh);
}

// bochscpu_backend.cc:352-410: one testcase on lane 0; the caller already ran
// Target.InsertTestcase against this backend (client.cc:102-111).
std::optional<TestcaseResult_t> GpuBackend_t::Run(const uint8_t *, const uint64_t) {
  const auto t0 = Clock::now();
  cur_ = 0;
  if (flush_lanes({0}) || upload_feed(1)) return std::nullopt;
  std::vector<LaneResult> out(1);
  if (!run_lanes({0}, &out, nullptr, false)) return std::nullopt;
  // the lane's final registers back into its view: GetReg after Run reads
  // them (the client's own code and Target.Restore may do so)
  LaneView &v = view(0);
  if (wtfgpu_read_gprs_list(ctx_, &cur_, 1, v.gpr)) return std::nullopt;
  v.regs_dirty = false;
  v.cr_known = 0;
  last_icount_ = out[0].icount;
  last_error_ = out[0].error;
  {  // run stats of this testcase (PrintRunStats)
    uint64_t nbytes = 0;
    uint32_t dcount = 0, ecount[2] = {0, 0};
    wtfgpu_read_bytes(ctx_, 0, 1, &nbytes);
    wtfgpu_read_dirty_counts(ctx_, 0, 1, &dcount);
    wtfgpu_read_edge_counts(ctx_, 0, 1, ecount);
    last_run_ = out[0];
    last_run_.bytes = nbytes;
    last_run_.dirty = std::min(dcount, overlay_pages_);
    last_run_.edges = ecount[0];
    last_run_.edges_new = ecount[1];
  }
  finish_coverage(1, nullptr, nullptr);  // Timedout revocation is the client's call (RevokeLastNewCoverage)
  stats_.total_ms += ms_since(t0);
  cur_ = 0;
  return out[0].result;
}

bool GpuBackend_t::LaneTrace(uint32_t Lane, std::vector<uint64_t> &Rips, bool &Truncated) {
  uint64_t N = 0;
  Rips.clear();
  if (wtfgpu_read_trace(ctx_, Lane, nullptr, 0, &N) != WTFGPU_OK) return false;
  Truncated = N > trace_cap_;
  Rips.resize(std::min<uint64_t>(N, trace_cap_));
  return wtfgpu_read_trace(ctx_, Lane, Rips.data(), Rips.size(), &N) == WTFGPU_OK;
}

bool GpuBackend_t::LaneTenet(uint32_t Lane, std::vector<uint8_t> &Bytes, bool &Truncated) {
  uint64_t N = 0;
  Bytes.clear();
  if (wtfgpu_read_tenet(ctx_, Lane, nullptr, 0, &N) != WTFGPU_OK) return false;
  Truncated = N > tenet_cap_;
  Bytes.resize(std::min<uint64_t>(N, tenet_cap_));
  return wtfgpu_read_tenet(ctx_, Lane, Bytes.data(), Bytes.size(), &N) == WTFGPU_OK;
}

bool GpuBackend_t::RunBatch(const Target_t &Target, const std::vector<std::pair<const uint8_t *, size_t>> &Testcases,
                            std::vector<LaneResult> &Out, ModuleSlots *Slots) {
  const auto t0 = Clock::now();
  const uint32_t n = (uint32_t)Testcases.size();
  if (n == 0 || n > nlanes_) return false;
  Out.assign(n, LaneResult{});
  // module state: each lane is reset right before its InsertTestcase, inside
  // the (parallel) insert loop (ModuleSlots::ResetLane)
  if (wtfgpu_restore(ctx_, 0, n)) return false;
  for (uint32_t l = 0; l < n; l++) reset_view(l);
  const auto tm = Clock::now();
  stats_.restore_ms += std::chrono::duration<double, std::milli>(tm - t0).count();
  // InsertTestcase per lane (client.cc:102), module state per lane
  std::vector<uint32_t> lanes(n);
  for (uint32_t l = 0; l < n; l++) lanes[l] = l;
  std::vector<uint8_t> insert_ok;
  insert_lanes(Target, lanes, Testcases, Slots, insert_ok);
  for (uint32_t l = 0; l < n; l++)
    if (!insert_ok[l]) view(l).result = Crash_t("insert-testcase-failed");
  const auto tu = Clock::now();
  stats_.module_ms += std::chrono::duration<double, std::milli>(tu - tm).count();
  if (flush_lanes(lanes) || upload_feed(n)) return false;
  stats_.upload_ms += ms_since(tu);
  stats_.insert_ms += ms_since(t0);
  if (!run_lanes(lanes, &Out, Slots, Slots != nullptr)) return false;
  {  // B_exec = instruction + data bytes, testcase bytes, 2 x 4096 per dirty page
    std::vector<uint64_t> nb(n);
    std::vector<uint32_t> dc(n);
    if (wtfgpu_read_bytes(ctx_, 0, n, nb.data()) == WTFGPU_OK &&
        wtfgpu_read_dirty_counts(ctx_, 0, n, dc.data()) == WTFGPU_OK)
      for (uint32_t l = 0; l < n; l++) stats_.alg_bytes += nb[l] + 2ull * 4096 * dc[l] + Testcases[l].second;
  }
  const auto tc = Clock::now();
  std::vector<uint32_t> timedout;
  for (uint32_t l = 0; l < n; l++)
    if (std::holds_alternative<Timedout_t>(Out[l].result)) timedout.push_back(l);
  finish_coverage(n, &Out, &timedout);
  const auto tr = Clock::now();
  stats_.coverage_ms += std::chrono::duration<double, std::milli>(tr - tc).count();
  // Target.Restore per lane (client.cc:145), then the device restore happens
  // at the start of the next batch (dirty-list reset)
  target_restore(Target, lanes, Slots);
  stats_.target_restore_ms += ms_since(tr);
  stats_.total_ms += ms_since(t0);
  stats_.batches++;
  stats_.testcases += n;
  return true;
}

void GpuBackend_t::insert_lanes(const Target_t &Target, const std::vector<uint32_t> &lanes,
                                const std::vector<std::pair<const uint8_t *, size_t>> &tcs, ModuleSlots *Slots,
                                std::vector<uint8_t> &ok) {
  Backend_t *saved = g_Backend;
  ok.assign(lanes.size(), 1);
  auto insert = [&](size_t i) {
    const uint32_t l = lanes[i];
    cur_ = l;
    if (Slots) {
      Slots->ResetLane(l);
      Slots->SwapIn(l);
    }
    const Target_t &T = Slots && Slots->Instances() ? Slots->Instances()->TargetOf(l) : Target;
    try {
      ok[i] = T.InsertTestcase(tcs[i].first, tcs[i].second);
    } catch (const HandlerFault_t &) {  // see service_hits
      view(l).handler_fault = true;
      ok[i] = 0;
    }
    if (Slots) Slots->SwapOut(l);
  };
  if (parallel_service(Slots)) {
    HostPool::Get().For(lanes.size(), 256, [&](size_t i) {
      g_Backend = this;
      insert(i);
    });
  } else {
    g_Backend = this;
    for (size_t i = 0; i < lanes.size(); i++) insert(i);
  }
  g_Backend = saved;
}

// Target.Restore per lane (client.cc:145)
void GpuBackend_t::target_restore(const Target_t &Target, const std::vector<uint32_t> &lanes, ModuleSlots *Slots) {
  Backend_t *saved = g_Backend;
  auto restore = [&](uint32_t l) {
    cur_ = l;
    if (Slots) Slots->SwapIn(l);
    (Slots && Slots->Instances() ? Slots->Instances()->TargetOf(l) : Target).Restore();
    if (Slots) Slots->SwapOut(l);
  };
  if (parallel_service(Slots)) {
    HostPool::Get().For(lanes.size(), 256, [&](size_t i) {
      g_Backend = this;
      restore(lanes[i]);
    });
  } else {
    g_Backend = this;
    for (uint32_t l : lanes) restore(l);
  }
  g_Backend = saved;
  cur_ = 0;
}

// Streaming form of finish_coverage: the finished lanes' new rips, attributed
// in the given order against the aggregate (bochscpu_backend.cc:501-504);
// timed-out lanes' are revoked (client.cc:122-125); the fresh ones join the
// device map. Their log bits are dropped (the lanes get new testcases next).
void GpuBackend_t::collect_coverage(const std::vector<uint32_t> &lanes, std::vector<LaneResult> &res,
                                    const uint64_t *pf_hdr) {
  const auto t0 = Clock::now();
  uint64_t total = 0;
  uint32_t ovf = 0;
  constexpr uint64_t kPrefetchCap = 1ull << 22;  // wtfgpu_prefetched_coverage's limit
  bool pf = pf_hdr && pf_hdr[0] <= kPrefetchCap;
  if (pf) {
    // the part's stopped lanes' sets, gathered behind the slice: only the
    // entries of `lanes` count; their sets are emptied as a read here would
    total = pf_hdr[0];
    ovf = (uint32_t)pf_hdr[1] & 1;
    if (cov_lanes_.size() < total) {
      cov_lanes_.resize(total);
      cov_rips_.resize(total);
    }
    pf = wtfgpu_prefetched_coverage(ctx_, cov_lanes_.data(), cov_rips_.data(), total) == WTFGPU_OK &&
         wtfgpu_clear_coverage_lanes(ctx_, lanes.data(), (uint32_t)lanes.size()) == WTFGPU_OK;
    if (pf && total) {
      if (cov_want_.size() < nlanes_) cov_want_.assign(nlanes_, 0);
      for (uint32_t l : lanes) cov_want_[l] = 1;
      uint64_t k = 0;
      for (uint64_t i = 0; i < total; i++)
        if (cov_want_[cov_lanes_[i]]) {
          cov_lanes_[k] = cov_lanes_[i];
          cov_rips_[k++] = cov_rips_[i];
        }
      for (uint32_t l : lanes) cov_want_[l] = 0;
      total = k;
    }
  }
  if (!pf) {
    total = 0;
    ovf = 0;
    // one call into buffers that persist (the sets empty when it all fits);
    // a larger result is read again at its size
    if (cov_lanes_.size() < (1u << 16)) {
      cov_lanes_.resize(1u << 16);
      cov_rips_.resize(1u << 16);
    }
    wtfgpu_collect_coverage_lanes(ctx_, lanes.data(), (uint32_t)lanes.size(), cov_lanes_.data(), cov_rips_.data(),
                                  cov_lanes_.size(), &total, &ovf);
    if (total > cov_lanes_.size()) {
      cov_lanes_.resize(total);
      cov_rips_.resize(total);
      wtfgpu_collect_coverage_lanes(ctx_, lanes.data(), (uint32_t)lanes.size(), cov_lanes_.data(), cov_rips_.data(),
                                    cov_lanes_.size(), &total, &ovf);
    }
  }
  const std::vector<uint32_t> &cl = cov_lanes_;
  const std::vector<uint64_t> &cr = cov_rips_;
  const auto t1 = Clock::now();
  stats_.covlog_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
  stats_.cov_entries += total;
  if (ovf && !cov_ovf_warned_) {
    cov_ovf_warned_ = true;
    fprintf(stderr, "wtfgpu: a lane's new-coverage set filled up (rips lost); raise the set size\n");
  }
  // the entries come back in no order: sorted by (lane, rip) and unique, each
  // lane's set is one run, found by binary search in the order given
  std::vector<std::pair<uint32_t, uint64_t>> &ent = cov_sorted_;
  ent.resize(total);
  for (uint64_t i = 0; i < total; i++) ent[i] = {cl[i], cr[i]};
  std::sort(ent.begin(), ent.end());
  ent.erase(std::unique(ent.begin(), ent.end()), ent.end());
  if (getenv("WTFGPU_COVLOG_TOP")) {  // diagnostic: which logged values keep coming back
    for (uint64_t i = 0; i < total; i++) covlog_count_[cr[i]]++;
    if (++covlog_calls_ % 64 == 0) {
      std::vector<std::pair<uint64_t, uint64_t>> v(covlog_count_.begin(), covlog_count_.end());
      std::sort(v.begin(), v.end(), [](auto &a, auto &b) { return a.second > b.second; });
      fprintf(stderr, "covlog top:");
      for (size_t i = 0; i < v.size() && i < 24; i++)
        fprintf(stderr, " %llx:%llu%s", (unsigned long long)v[i].first, (unsigned long long)v[i].second,
                aggregate_.count(v[i].first) ? "*" : "");
      fprintf(stderr, " (%zu values)\n", v.size());
    }
  }
  std::vector<uint64_t> fresh;
  last_new_coverage_.clear();
  // one lane's run of entries, attributed against the aggregate (lanes in order)
  auto attribute = [&](uint32_t l, size_t at) {
    const bool revoke = std::holds_alternative<Timedout_t>(res[l].result);
    for (; at < ent.size() && ent[at].first == l; at++) {
      const uint64_t rip = ent[at].second;
      if (full_coverage_) {  // parity mode: the lane's whole rip set, nothing committed
        res[l].new_coverage.push_back(rip);
        continue;
      }
      if (aggregate_.count(rip)) continue;
      res[l].new_coverage.push_back(rip);
      if (revoke) continue;
      aggregate_.insert(rip);
      fresh.push_back(rip);
    }
    return at;
  };
  if (std::is_sorted(lanes.begin(), lanes.end())) {
    // the entries' lane order is the given order: one pass over the runs
    for (size_t at = 0; at < ent.size();) at = attribute(ent[at].first, at);
  } else {
    for (uint32_t l : lanes) {
      const auto it = std::lower_bound(ent.begin(), ent.end(), std::pair<uint32_t, uint64_t>{l, 0});
      if (it != ent.end() && it->first == l) attribute(l, (size_t)(it - ent.begin()));
    }
  }
  commit_fresh(fresh);
  stats_.attrib_ms += ms_since(t1);
}

uint32_t GpuBackend_t::FreeLanes() const {
  if (busy_.empty()) return parts_n() > 1 ? nlanes_ / 2 : nlanes_;
  const Part &P = parts_[next_part_];
  if (P.launched) return P.hi - P.lo;  // its running lanes may all finish: an upper bound
  return (uint32_t)P.free.size();
}

// Streaming parts: one (every lane, synchronous) or two halves on their own
// queues, pipelined: StreamStep harvests and refills one half while the
// other half's slice runs on the GPU (WTFGPU_STREAM_PARTS=1 turns it off).
uint32_t GpuBackend_t::parts_n() const {
  if (!parts_.empty()) return (uint32_t)parts_.size();
  const char *e = getenv("WTFGPU_STREAM_PARTS");
  const uint32_t want = e ? (uint32_t)atoi(e) : 2;
  return (want >= 2 && nlanes_ >= 256 && nlanes_ % 128 == 0) ? 2 : 1;
}

// One streaming step on the next part: its finished slice is harvested (when
// pipelined), its free lanes get testcases from `In` (restore +
// InsertTestcase + uploads), and its occupied lanes start one slice of
// `Slice` wave-steps (without the pipeline: harvested in the same call).
bool GpuBackend_t::StreamStep(const Target_t &Target, const std::vector<StreamTestcase_t> &In, uint64_t Slice,
                              std::vector<StreamResult_t> &Out, ModuleSlots *Slots, size_t *Taken) {
  const auto t0 = Clock::now();
  if (Taken) *Taken = 0;
  if (busy_.empty()) {
    busy_.assign(nlanes_, 0);
    tag_.assign(nlanes_, 0);
    tc_bytes_.assign(nlanes_, 0);
    lres_.assign(nlanes_, LaneResult{});
    lres_stale_.assign(nlanes_, 0);
    const uint32_t n = parts_n();
    parts_.assign(n, Part{});
    for (uint32_t p = 0; p < n; p++) {
      Part &Q = parts_[p];
      Q.lo = (uint32_t)((uint64_t)nlanes_ * p / n);
      Q.hi = (uint32_t)((uint64_t)nlanes_ * (p + 1) / n);
      Q.free.resize(Q.hi - Q.lo);
      for (uint32_t l = Q.lo; l < Q.hi; l++) Q.free[l - Q.lo] = l;
    }
    // every lane idle until it gets a testcase
    std::vector<uint32_t> all(nlanes_);
    for (uint32_t l = 0; l < nlanes_; l++) all[l] = l;
    if (wtfgpu_stop(ctx_, all.data(), nlanes_, WTFGPU_EXIT_IDLE)) return false;
  }
  const bool pipelined = parts_.size() > 1;
  const uint32_t pi = next_part_;
  next_part_ = (next_part_ + 1) % (uint32_t)parts_.size();
  Part &P = parts_[pi];
  if (pipelined && wtfgpu_select_queue(ctx_, pi)) return false;
  if (pipelined && P.launched && !harvest_part(P, Target, Out, Slots)) return false;
  const auto ti = Clock::now();
  stats_.harvest_ms += std::chrono::duration<double, std::milli>(ti - t0).count();
  // ---- refill
  std::vector<uint32_t> fresh;
  std::vector<std::pair<const uint8_t *, size_t>> tcs;
  fresh.reserve(std::min<size_t>(In.size(), P.hi - P.lo));
  tcs.reserve(fresh.capacity());
  {  // the lowest free lanes, in order
    const size_t take = std::min(In.size(), P.free.size());
    fresh.assign(P.free.begin(), P.free.begin() + (std::ptrdiff_t)take);
    P.free.erase(P.free.begin(), P.free.begin() + (std::ptrdiff_t)take);
    tcs.resize(take);
    for (size_t i = 0; i < take; i++) tcs[i] = {In[i].data, In[i].size};
  }
  if (Taken) *Taken = fresh.size();
  stats_.fresh_ms += ms_since(ti);
  if (!fresh.empty()) {
    if (wtfgpu_restore_lanes(ctx_, fresh.data(), (uint32_t)fresh.size())) return false;
    stats_.restore_dev_ms += ms_since(ti);
    // a prepared insert (Target_t::PrepareInsert) the backend takes is applied
    // here, with the lane's module state reset as before an InsertTestcase;
    // the other lanes call InsertTestcase below
    std::vector<uint8_t> prepared(fresh.size(), 0);
    HostPool::Get().For(fresh.size(), 256, [&](size_t i) {
      const uint32_t l = fresh[i];
      // a view the host touched goes back to the initial state; an untouched
      // one still is in it (the common case: no host handler ran on the lane)
      if (touched_[l]) reset_view(l);
      pf_[l] = PrepFeed{};
      busy_[l] = 1;
      tag_[l] = In[i].tag;
      tc_bytes_[l] = In[i].size;
      lres_stale_[l] = 1;  // its last result may not be consumed yet (this call's Out)
      const StreamTestcase_t &T = In[i];
      switch (T.prep) {
        case PreparedInsert_t::Call: return;
        case PreparedInsert_t::Failed: view(l).result = Crash_t("insert-testcase-failed"); break;
        case PreparedInsert_t::Nothing: break;
        case PreparedInsert_t::Feed:  // SetFeed would refuse it: InsertTestcase keeps its host path
          if (!feed_action_ || T.prep_size > kFeedRegion) return;
          pf_[l] = PrepFeed{T.prep_data, (uint32_t)T.prep_size, 1, 0};
          break;
        case PreparedInsert_t::Insert:  // as SetInsert
          if (!insert_action_ || T.size + 4 > kFeedRegion) return;
          pf_[l] = PrepFeed{T.data, (uint32_t)T.size, 1, 1};
          break;
      }
      if (Slots) Slots->ResetLane(l);
      prepared[i] = 1;
    });
    recycle_arenas();  // reset_view's drop_staged ran inside the loop
    const auto tm = Clock::now();
    stats_.restore_ms += std::chrono::duration<double, std::milli>(tm - ti).count();
    std::vector<uint32_t> call;
    std::vector<std::pair<const uint8_t *, size_t>> call_tcs;
    for (size_t i = 0; i < fresh.size(); i++)
      if (!prepared[i]) {
        call.push_back(fresh[i]);
        call_tcs.push_back(tcs[i]);
      }
    stats_.prepared += fresh.size() - call.size();
    if (!call.empty()) {
      std::vector<uint8_t> ok;
      insert_lanes(Target, call, call_tcs, Slots, ok);
      for (size_t i = 0; i < call.size(); i++)
        if (!ok[i]) view(call[i]).result = Crash_t("insert-testcase-failed");
    }
    const auto tu = Clock::now();
    stats_.module_ms += std::chrono::duration<double, std::milli>(tu - tm).count();
    if (flush_lanes(call)) return false;
    if (feed_action_ || insert_action_) {
      const auto tf = Clock::now();
      const size_t n = fresh.size();
      std::vector<uint64_t> off(n + 1, 0);
      std::vector<uint8_t> has(n);
      HostPool::Get().For(n, 1024, [&](size_t i) {  // prepared feeds, else a view's SetFeed / SetInsert bytes
        const uint32_t l = fresh[i];
        const PrepFeed &f = pf_[l];
        const bool t = !f.has && touched_[l];
        off[i + 1] = f.has ? f.len + (f.ins ? 4 : 0) : t ? views_[l].feed.size() : 0;
        has[i] = f.has || (t && views_[l].has_feed);
      });
      for (size_t i = 0; i < n; i++) off[i + 1] += off[i];
      // packed into the part's pinned buffer on all host threads: one DMA
      if (off[n] > P.pin_cap) {
        if (P.pin) wtfgpu_host_free(ctx_, P.pin);
        P.pin = nullptr;
        P.pin_cap = std::max<uint64_t>(off[n] * 2, 1 << 20);
        void *p = nullptr;
        if (wtfgpu_host_alloc(ctx_, P.pin_cap, &p)) return false;
        P.pin = (uint8_t *)p;
      }
      HostPool::Get().For(n, 256, [&](size_t i) {
        const uint32_t l = fresh[i];
        const PrepFeed &f = pf_[l];
        uint8_t *o = P.pin + off[i];
        if (f.has) {
          if (f.ins) {
            memcpy(o, &f.len, 4);
            o += 4;
          }
          if (f.len) memcpy(o, f.p, f.len);
        } else if (touched_[l] && !views_[l].feed.empty()) {
          memcpy(o, views_[l].feed.data(), views_[l].feed.size());
        }
      });
      if (wtfgpu_set_feed_lanes(ctx_, fresh.data(), (uint32_t)n, off.data(), has.data(), P.pin, off[n]))
        return false;
      stats_.up_feed_ms += ms_since(tf);
    }
    if (!stop_prestopped(fresh)) return false;
    stats_.upload_ms += ms_since(tu);
    stats_.testcases += fresh.size();
  }
  stats_.insert_ms += ms_since(ti);
  // ---- one slice over the part's occupied lanes
  const auto to = Clock::now();
  if (!fresh.empty()) {  // occupied: the lanes still running plus the refilled ones
    std::vector<uint32_t> occ(P.occ.size() + fresh.size());
    std::merge(P.occ.begin(), P.occ.end(), fresh.begin(), fresh.end(), occ.begin());
    P.occ.swap(occ);
  }
  stats_.occ_ms += ms_since(to);
  if (!P.occ.empty()) {
    const auto tk = Clock::now();
    if (wtfgpu_run_async(ctx_, P.lo, P.hi - P.lo, Slice ? Slice : 4096)) return false;
    P.pf = pipelined && prefetch_part(P);
    stats_.run_ms += ms_since(tk);
    P.launched = true;
    if (!pipelined && !harvest_part(P, Target, Out, Slots)) return false;
  }
  stats_.total_ms += ms_since(t0);
  return true;
}

// The slice's read-back queued behind it on the part's queue (exits, byte and
// dirty counts, StopWithArgs arguments, the stopped lanes' coverage), into
// pinned buffers the harvest reads after wtfgpu_run_wait without a device
// call of its own. false: nothing queued (the harvest reads them itself).
bool GpuBackend_t::prefetch_part(Part &P) {
  const uint32_t count = P.hi - P.lo;
  auto grow = [&](auto *&p, uint64_t bytes) {
    if (p) return true;
    void *q = nullptr;
    if (wtfgpu_host_alloc(ctx_, bytes, &q)) return false;
    p = (std::remove_reference_t<decltype(p)>)q;
    return true;
  };
  if (P.ex_cap < count) {
    if (P.ex) wtfgpu_host_free(ctx_, P.ex);
    P.ex = nullptr;
    P.ex_cap = 0;
    if (!grow(P.ex, (uint64_t)count * sizeof(wtfgpu_exit_t))) return false;
    P.ex_cap = count;
  }
  const bool args = !args_results_.empty();
  if (!grow(P.nb, (uint64_t)count * 8) || !grow(P.dc, (uint64_t)count * 4) || !grow(P.cov_hdr, 16) ||
      (args && !grow(P.sargs, (uint64_t)count * 48)))
    return false;
  if (wtfgpu_prefetch_results(ctx_, P.lo, count, P.ex, P.nb, P.dc, args ? P.sargs : nullptr) != WTFGPU_OK)
    return false;
  P.pf_cov = !full_coverage_ && wtfgpu_prefetch_coverage(ctx_, P.lo, count, P.cov_hdr) == WTFGPU_OK;
  return true;
}

// The part's slice: wait for it, classify the exits, service breakpoint hits
// (those lanes resume in the next slice), and harvest the finished lanes
// (results, coverage attribution in lane order, Target.Restore).
bool GpuBackend_t::harvest_part(Part &P, const Target_t &Target, std::vector<StreamResult_t> &Out,
                                ModuleSlots *Slots) {
  const auto tw = Clock::now();
  wtfgpu_run_stats_t rs{};
  if (wtfgpu_run_wait(ctx_, &rs)) return false;
  const auto te = Clock::now();
  stats_.run_ms += std::chrono::duration<double, std::milli>(te - tw).count();
  account_run(rs);
  P.launched = false;
  const uint32_t first = P.lo, count = P.hi - P.lo;
  // the results handed out for these lanes' previous testcases were consumed
  // before this call: clear them (capacity kept) before this slice's go in
  HostPool::Get().For(P.occ.size(), 1024, [&](size_t i) {
    const uint32_t l = P.occ[i];
    if (!lres_stale_[l]) return;
    lres_stale_[l] = 0;
    LaneResult &r = lres_[l];
    r.result = Ok_t();
    r.error = false;
    r.handler_fault = false;
    r.exit_status = 0;
    r.icount = 0;
    r.rip = 0;
    r.new_coverage.clear();
  }, P.occ.size() >= 8192);
  const bool pf = P.pf;  // the exits (and counts, arguments, coverage count) are in P's pinned buffers
  P.pf = false;
  if (!pf) {
    if (P.ex_cap < count) {
      if (P.ex) wtfgpu_host_free(ctx_, P.ex);
      P.ex = nullptr;
      P.ex_cap = 0;
      void *p = nullptr;
      if (wtfgpu_host_alloc(ctx_, (uint64_t)count * sizeof(wtfgpu_exit_t), &p)) return false;
      P.ex = (wtfgpu_exit_t *)p;
      P.ex_cap = count;
    }
    if (wtfgpu_read_exits(ctx_, first, count, P.ex)) return false;
  }
  std::vector<uint8_t> done(count, 0);
  std::vector<uint32_t> hits;
  if (!classify(P.occ, first, P.ex, done, &lres_, hits, pf ? P.sargs : nullptr)) return false;
  stats_.exits_ms += ms_since(te);
  if (!hits.empty() && !service_hits(hits, first, done, Slots, Slots != nullptr)) return false;
  std::vector<uint32_t> finished;
  if (!fill_results(P.occ, first, P.ex, done, &lres_, &finished)) return false;
  if (finished.empty()) return true;
  const auto tc = Clock::now();
  if (pf) {  // B_exec = instruction + data bytes, testcase bytes, 2 x 4096 per dirty page
    uint64_t b = 0;
    for (uint32_t l : finished) b += P.nb[l - first] + 2ull * 4096 * P.dc[l - first] + tc_bytes_[l];
    stats_.alg_bytes += b;
  } else {
    uint32_t lo = finished.front() & ~63u, hi = finished.back() + 1;
    std::vector<uint64_t> nb(hi - lo);
    std::vector<uint32_t> dc(hi - lo);
    if (wtfgpu_read_bytes(ctx_, lo, hi - lo, nb.data()) == WTFGPU_OK &&
        wtfgpu_read_dirty_counts(ctx_, lo, hi - lo, dc.data()) == WTFGPU_OK)
      for (uint32_t l : finished) stats_.alg_bytes += nb[l - lo] + 2ull * 4096 * dc[l - lo] + tc_bytes_[l];
  }
  stats_.bytes_ms += ms_since(tc);
  collect_coverage(finished, lres_, pf && P.pf_cov ? P.cov_hdr : nullptr);
  const auto tr = Clock::now();
  stats_.coverage_ms += std::chrono::duration<double, std::milli>(tr - tc).count();
  target_restore(Target, finished, Slots);
  stats_.target_restore_ms += ms_since(tr);
  const auto tout = Clock::now();
  const size_t base = Out.size();
  Out.resize(base + finished.size());
  for (size_t i = 0; i < finished.size(); i++) {
    const uint32_t l = finished[i];
    Out[base + i] = StreamResult_t{tag_[l], &lres_[l]};
    busy_[l] = 0;  // not runnable until refilled (a finished lane keeps its exit status)
  }
  {  // the finished lanes leave the occupied list for the free one (all ascending)
    std::vector<uint32_t> occ(P.occ.size()), fr(P.free.size() + finished.size());
    occ.resize(std::set_difference(P.occ.begin(), P.occ.end(), finished.begin(), finished.end(), occ.begin()) -
               occ.begin());
    std::merge(P.free.begin(), P.free.end(), finished.begin(), finished.end(), fr.begin());
    P.occ.swap(occ);
    P.free.swap(fr);
  }
  stats_.out_ms += ms_since(tout);
  stats_.batches++;
  return true;
}

void GpuBackend_t::ResetCoverage() {
  aggregate_.clear();
  last_new_coverage_.clear();
  wtfgpu_reset_coverage(ctx_);
}

std::string GpuBackend_t::StatsJson() const {
  char b[2048];
  snprintf(b, sizeof(b),
           "{\"kind\":\"gpu\",\"group_steps\":%llu,\"rounds\":%llu,\"breakpoint_hits\":%llu,\"kernel_launches\":%llu,"
           "\"kernel_ms\":%.3f,\"service_ms\":%.3f,\"total_ms\":%.3f,\"page_fetches\":%llu,"
           "\"prefetched_pages\":%llu,\"stack_windows\":%llu,\"staged_pages\":%llu,\"bulk_ms\":%.3f,\"prefetch_ms\":%.3f,"
           "\"handler_ms\":%.3f,\"fetch_ms\":%.3f,\"flush_ms\":%.3f,\"insert_ms\":%.3f,\"coverage_ms\":%.3f,"
           "\"target_restore_ms\":%.3f,\"alg_bytes\":%llu,\"restore_ms\":%.3f,\"module_ms\":%.3f,"
           "\"upload_ms\":%.3f,\"bytes_ms\":%.3f,\"covlog_ms\":%.3f,\"attrib_ms\":%.3f,\"cov_entries\":%llu,"
           "\"run_ms\":%.3f,\"exits_ms\":%.3f,\"regs_ms\":%.3f,\"err_unimpl\":%llu,\"err_overlay\":%llu,"
           "\"err_other\":%llu,\"err_handler\":%llu,\"last_unimpl_op\":%llu,\"last_unimpl_rip\":%llu}",
           (unsigned long long)stats_.group_steps, (unsigned long long)stats_.rounds,
           (unsigned long long)stats_.breakpoint_hits, (unsigned long long)stats_.kernel_launches, stats_.kernel_ms,
           stats_.service_ms, stats_.total_ms, (unsigned long long)stats_.page_fetches,
           (unsigned long long)stats_.prefetched_pages, (unsigned long long)stats_.stack_windows,
           (unsigned long long)stats_.staged_pages, stats_.bulk_ms, stats_.prefetch_ms, stats_.handler_ms,
           stats_.fetch_ms, stats_.flush_ms, stats_.insert_ms, stats_.coverage_ms, stats_.target_restore_ms,
           (unsigned long long)stats_.alg_bytes, stats_.restore_ms, stats_.module_ms, stats_.upload_ms,
           stats_.bytes_ms, stats_.covlog_ms, stats_.attrib_ms, (unsigned long long)stats_.cov_entries,
           stats_.run_ms, stats_.exits_ms, stats_.regs_ms, (unsigned long long)stats_.err_unimpl.load(),
           (unsigned long long)stats_.err_overlay.load(), (unsigned long long)stats_.err_other.load(),
           (unsigned long long)stats_.err_handler.load(), (unsigned long long)stats_.last_unimpl_op.load(), (unsigned long long)stats_.last_unimpl_rip.load());
  std::string r(b);
  r.pop_back();
  snprintf(b, sizeof(b), ",\"up_prep_ms\":%.3f,\"up_regs_ms\":%.3f,\"up_apply_ms\":%.3f,\"up_feed_ms\":%.3f,"
           "\"restore_dev_ms\":%.3f,\"out_ms\":%.3f,\"fresh_ms\":%.3f,\"occ_ms\":%.3f,\"harvest_ms\":%.3f,"
           "\"prepared\":%llu",
           stats_.up_prep_ms, stats_.up_regs_ms, stats_.up_apply_ms, stats_.up_feed_ms, stats_.restore_dev_ms,
           stats_.out_ms, stats_.fresh_ms, stats_.occ_ms, stats_.harvest_ms, (unsigned long long)stats_.prepared);
  r += b;
  r += ",\"unimpl_ops\":" + stats_.unimpl_ops.json();
  r += ",\"unimpl_raw\":" + stats_.unimpl_ops.raw_json();
  b[0] = 0;
  r += b;
  r += ",\"fetch_by_bp\":{";
  bool first = true;
  for (const auto &[bp, n] : fetch_by_bp_) {
    char e[64];
    snprintf(e, sizeof(e), "%s\"%#llx\":%llu", first ? "" : ",", (unsigned long long)bp, (unsigned long long)n);
    r += e;
    first = false;
  }
  return r + "}}";
}

// Coverage index space: every executable leaf page reachable
// from the snapshot cr3 gets a slot in the device coverage map; identical on
// every GPU, so the maps can be merged with a MAX all-reduce.
bool GpuBackend_t::set_code_pages() {
  const std::vector<uint64_t> vpns = ExecutablePages(dump_, initial_.Cr3);
  code_vpns_.clear();
  code_vpns_.insert(vpns.begin(), vpns.end());
  if (vpns.empty()) return true;
  return wtfgpu_set_code_pages(ctx_, vpns.data(), (uint32_t)vpns.size()) == WTFGPU_OK;
}

bool GpuBackend_t::CoverageMap(uint8_t **Map, uint64_t *Bytes, bool *Device) {
  void *p = nullptr;
  if (wtfgpu_coverage_device_map(ctx_, &p, Bytes) != WTFGPU_OK) return false;
  *Map = (uint8_t *)p;
  *Device = true;
  return true;
}

// Rips other shards set in the merged map (the engine reports what changed
// since its last look; its own commits are not reported) join the aggregate.
size_t GpuBackend_t::AbsorbCoverageMap() {
  uint64_t n = 0;
  if (wtfgpu_coverage_absorb(ctx_, nullptr, 0, &n) != WTFGPU_OK || n == 0) return 0;
  std::vector<uint64_t> rips(n);
  if (wtfgpu_coverage_absorb(ctx_, rips.data(), n, &n) != WTFGPU_OK) return 0;
  size_t added = 0;
  for (uint64_t i = 0; i < n && i < rips.size(); i++) added += aggregate_.insert(rips[i]).second;
  return added;
}

// New aggregate values go to the device map (code pages) or its extra set
// (wtfgpu_commit_coverage); the ones outside the map are also kept for the
// cross-shard overflow merge.
void GpuBackend_t::commit_fresh(const std::vector<uint64_t> &fresh) {
  if (fresh.empty()) return;
  for (uint64_t v : fresh)
    if (!code_vpns_.count(v >> 12)) extra_new_.push_back(v);
  wtfgpu_commit_coverage(ctx_, fresh.data(), fresh.size());
}

void GpuBackend_t::TakeNewExtra(std::vector<uint64_t> &Out) {
  Out.swap(extra_new_);
  extra_new_.clear();
}

// Other shards' values outside the map join the aggregate and the device set
// (so lanes stop logging them); returns how many were new here.
size_t GpuBackend_t::AbsorbExtra(const std::vector<uint64_t> &All) {
  std::vector<uint64_t> add;
  for (uint64_t v : All)
    if (aggregate_.insert(v).second) add.push_back(v);
  if (!add.empty()) wtfgpu_commit_coverage(ctx_, add.data(), add.size());
  return add.size();
}

}  // namespace wtfgpu_host
