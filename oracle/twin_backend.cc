// twin_backend.cc — TEST INFRASTRUCTURE ONLY: the CPU twin of the gpu backend.
//
// A Backend_t over the scalar oracle (x86_oracle.c), running testcases one
// after the other exactly as wtf's client loop drives bochscpu
// (RunTestcaseAndRestore, client.cc:88-180; BochscpuBackend_t::Run /
// Restore, bochscpu_backend.cc:352-410, 730-797). It runs the same fuzzer
// modules and the same batched runner as `wtfgpu`, so per-testcase results,
// retired counts, final registers and coverage sets can be compared lane by
// lane (tests/test_gpu_tlv.py), and it is the CPU baseline of the TLV bench
// (one process per host core, bench.py). The product never links this file.
#include "../wtf_amd/host/unimpl_hist.h"
#include "../wtf_amd/host/module_instances.h"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <unordered_map>

#include "../include/wtfgpu.h"
#include "../wtf_amd/host/runner.h"
#include "../wtf_amd/host/remote.h"
#include "../wtf_amd/host/wtf_api.h"
#include "x86_oracle.h"
#include "../wtf_amd/host/kdmp.h"
#include "../wtf_amd/host/blake3_lite.h"
#include "../wtf_amd/host/net_exchange.h"

#include <memory>

using namespace wtfgpu_host;


namespace {
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
    default: return -1;
  }
}
}  // namespace

class TwinBackend_t final : public Backend_t, public Executor_t {
  orc_machine *m_ = nullptr;
  KernelDump dump_;
  CpuState_t initial_{};
  wtfgpu_regs_t regs0_{};
  std::unordered_map<uint64_t, BreakpointHandler_t> bps_;
  std::optional<TestcaseResult_t> result_;
  uint64_t seed_ = 0;
  struct Staged {
    std::vector<uint8_t> data, orig;
  };
  mutable std::unordered_map<uint64_t, Staged> staged_;
  std::unordered_set<uint64_t> aggregate_;
  std::unordered_set<Gva_t> last_new_;
  uint64_t retired_total_ = 0;
  uint32_t trace_cap_ = 0;                      // rip traces (EnableTrace)
  std::vector<std::vector<uint64_t>> traces_;   // per testcase of the last RunBatch
  uint64_t inject_ = ~0ull;  // page to #PF after the current handler
  // coverage map over the executable-page slots (ExecutablePages, as the gpu
  // backend builds it) and its shadow, for the shard merge
  std::unordered_map<uint64_t, uint32_t> slot_;
  std::vector<uint64_t> slot_vpn_;
  std::vector<uint8_t> map_, shadow_;
  void map_set(uint64_t rip) {
    auto it = slot_.find(rip >> 12);
    if (it == slot_.end()) {  // outside the map: the overflow list other shards gather
      extra_new_.push_back(rip);
      return;
    }
    const uint64_t at = (uint64_t)it->second * 4096 + (rip & 0xfff);
    map_[at] = shadow_[at] = 1;
  }

  wtfgpu_regs_t regs() const {
    wtfgpu_regs_t r;
    orc_get_regs(m_, &r);
    return r;
  }
  void flush() {
    for (auto &[gpfn, s] : staged_)
      if (s.data != s.orig) orc_write_phys(m_, gpfn << 12, s.data.data(), 4096);
    staged_.clear();
  }

 public:
  ~TwinBackend_t() override {
    if (getenv("WTF_UNIMPL_HIST")) fprintf(stderr, "unimpl_ops %s\n", unimpl_.json(64).c_str());
    if (m_) orc_destroy(m_);
  }
  bool Initialize(const Options_t &Opts, const CpuState_t &CpuState) override {
    if (!dump_.Parse(Opts.DumpPath.string())) return false;
    slot_vpn_ = ExecutablePages(dump_, CpuState.Cr3);
    for (uint32_t i = 0; i < slot_vpn_.size(); i++) slot_.emplace(slot_vpn_[i], i);
    map_.assign(slot_vpn_.size() * 4096, 0);
    shadow_.assign(map_.size(), 0);
    m_ = orc_create();
    for (auto &[gpfn, page] : dump_.Pages()) orc_add_page(m_, gpfn, page);
    if (Opts.Limit) orc_set_limit(m_, Opts.Limit);
    orc_set_edges(m_, Opts.Edges ? 1 : 0);
    return Restore(CpuState);
  }
  // bochscpu_backend.cc:352-410 (+ the handler dispatch of :476-548)
  std::optional<TestcaseResult_t> Run(const uint8_t *, const uint64_t) override {
    flush();
    engine_error_ = false;
    handler_fault_ = false;
    int skip = 0;
    for (;;) {
      wtfgpu_exit_t e{};
      orc_run(m_, skip, &e);
      skip = 0;
      if (e.status == WTFGPU_EXIT_BREAKPOINT) {
        const uint64_t rip0 = regs().rip;
        BreakpointHandler_t handler = nullptr;
        if (route_) {
          handler = route_->HandlerOf(route_lane_, rip0);  // the lane's module copy (module_instances.h)
        } else {
          const auto it = bps_.find(rip0);
          if (it != bps_.end()) handler = it->second;
        }
        inject_ = ~0ull;
        try {
          if (handler) handler(this);
        } catch (const HandlerFault_t &) {  // U43: the handler ends at the failed access, the testcase as an engine error
          flush();
          result_ = Crash_t();
          engine_error_ = true;
          handler_fault_ = true;
          break;
        }
        flush();
        if (result_) break;
        skip = regs().rip == rip0;  // U10: a moved rip cancels the hooked instruction
        if (inject_ != ~0ull) {  // PageFaultsMemoryIfNeeded: #PF(Write|User) before the instruction
          if (!orc_inject_fault(m_, WTFGPU_VEC_PF, ErrorWrite | ErrorUser, inject_)) {
            result_ = Crash_t();  // no IDT to take it: the triple fault bochs would stop on
            break;
          }
          skip = 0;
        }
        if (!skip) orc_tenet_event(m_);  // Tenet: the handler moved rip (or injected a #PF)
        continue;
      }
      switch (e.status) {
        case WTFGPU_EXIT_TIMEOUT: result_ = Timedout_t(); break;
        case WTFGPU_EXIT_INT3:
        case WTFGPU_EXIT_HLT: result_ = Crash_t(); break;
        case WTFGPU_EXIT_CR3: result_ = Cr3Change_t(); break;
        case WTFGPU_EXIT_FAULT: result_ = FaultToResult(e.vector, e.error, e.rip, e.addr, e.opcode); break;
        default:  // outside the engine subset: an engine error, not a target crash
          result_ = Crash_t();
          engine_error_ = true;
          if (e.status == WTFGPU_EXIT_UNIMPLEMENTED) {
            unimpl_.add(e.opcode);
            if (getenv("WTF_UNIMPL_RAW")) fprintf(stderr, "unimpl_raw %08x rip %llx\n", e.opcode, (unsigned long long)e.rip);
          }
          break;
      }
      break;
    }
    // coverage of this testcase against the aggregate (bochscpu_backend.cc:501-504)
    std::vector<uint64_t> cov(orc_coverage(m_, nullptr, 0));
    orc_coverage(m_, cov.data(), cov.size());
    last_new_.clear();
    if (full_) aggregate_.clear();
    for (uint64_t r : cov)
      if (aggregate_.insert(r).second) last_new_.insert(Gva_t(r));
    if (!full_)
      for (const Gva_t &g : last_new_) map_set(g.U64());
    retired_total_ += orc_icount(m_);
    return result_;
  }
  bool Restore(const CpuState_t &CpuState) override {
    initial_ = CpuState;
    regs0_ = RegsFromCpuState(CpuState);
    orc_restore(m_, &regs0_);
    staged_.clear();
    result_.reset();
    seed_ = CpuState.Seed;
    return true;
  }
  void Stop(const TestcaseResult_t &Res) override { result_ = Res; }
  void SetLimit(const uint64_t Limit) override { orc_set_limit(m_, Limit); }
  uint64_t GetReg(const Registers_t Reg) override {
    const wtfgpu_regs_t r = regs();
    const int i = gpr_index(Reg);
    if (i >= 0) return r.gpr[i];
    if (Reg == Registers_t::Rip) return r.rip;
    if (Reg == Registers_t::Rflags) return r.rflags;
    if (Reg == Registers_t::Cr3) return r.cr3;
    if (Reg == Registers_t::Cr2) return r.cr2;
    return 0;
  }
  uint64_t SetReg(const Registers_t Reg, const uint64_t Value) override {
    wtfgpu_regs_t r = regs();
    const int i = gpr_index(Reg);
    if (i >= 0) r.gpr[i] = Value;
    else if (Reg == Registers_t::Rip) r.rip = Value;
    else if (Reg == Registers_t::Rflags) r.rflags = Value;
    else return Value;
    orc_set_regs(m_, &r);
    return Value;
  }
  uint64_t Rdrand() override;
  bool SetBreakpoint(const Gva_t Gva, const BreakpointHandler_t Handler) override {
    if (ModuleInstances *I = ModuleInstances::Registering()) {  // a module copy's Init
      I->AddHandler(Gva.U64(), Handler);
      if (I->RegisteringIndex() > 0) return bps_.count(Gva.U64()) != 0;
    }
    if (bps_.count(Gva.U64())) return false;
    bps_[Gva.U64()] = Handler;
    std::vector<uint64_t> v;
    for (auto &kv : bps_) v.push_back(kv.first);
    return orc_set_breakpoints(m_, v.data(), (uint32_t)v.size()) == 0;
  }
  using Backend_t::SetBreakpoint;
  bool DirtyGpa(const Gpa_t) override { return true; }
  bool VirtTranslate(const Gva_t Gva, Gpa_t &Gpa, const MemoryValidate_t) const override {
    // the staged pages may hold page-table edits not yet flushed: walk them
    uint64_t table = regs().cr3 & 0x000ffffffffff000ull;
    const uint64_t va = Gva.U64();
    for (int level = 3; level >= 0; level--) {
      uint64_t e;
      memcpy(&e, PhysTranslate(Gpa_t(table + ((va >> (12 + 9 * level)) & 0x1ff) * 8)), 8);
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
  uint8_t *PhysTranslate(const Gpa_t Gpa) const override {
    const uint64_t gpfn = Gpa.U64() >> 12;
    auto it = staged_.find(gpfn);
    if (it == staged_.end()) {
      Staged s;
      s.data.resize(4096);
      orc_read_phys(m_, gpfn << 12, s.data.data(), 4096);
      s.orig = s.data;
      it = staged_.emplace(gpfn, std::move(s)).first;
    }
    return it->second.data.data() + (Gpa.U64() & 0xfff);
  }
  // bochscpu_backend.cc:902-999: the first page of the range that does not
  // translate gets a #PF injected once the handler returns
  bool PageFaultsMemoryIfNeeded(const Gva_t Gva, const uint64_t Size) override {
    for (uint64_t a = Gva.U64() & ~0xfffull; a < Gva.U64() + Size; a += 0x1000) {
      Gpa_t G;
      if (!VirtTranslate(Gva_t(a), G, MemoryValidate_t::ValidateRead)) {
        inject_ = a;
        return true;
      }
    }
    return false;
  }
  const std::unordered_set<Gva_t> &LastNewCoverage() const override { return last_new_; }
  bool RevokeLastNewCoverage() override {
    for (const Gva_t &g : last_new_) {
      aggregate_.erase(g.U64());
      auto it = slot_.find(g.U64() >> 12);
      if (it != slot_.end()) map_[(uint64_t)it->second * 4096 + (g.U64() & 0xfff)] = shadow_[(uint64_t)it->second * 4096 + (g.U64() & 0xfff)] = 0;
    }
    last_new_.clear();
    return true;
  }

  // ---- Executor_t: RunTestcaseAndRestore per testcase (client.cc:88-180)
  Backend_t *AsBackend() override { return this; }
  uint32_t Lanes() const override { return 1u << 30; }
  void ResetCoverage() override {
    aggregate_.clear();
    last_new_.clear();
    std::fill(map_.begin(), map_.end(), 0);
    std::fill(shadow_.begin(), shadow_.end(), 0);
  }
  bool CoverageMap(uint8_t **Map, uint64_t *Bytes, bool *Device) override {
    *Map = map_.data();
    *Bytes = map_.size();
    *Device = false;
    return true;
  }
  void TakeNewExtra(std::vector<uint64_t> &Out) override {
    Out.swap(extra_new_);
    extra_new_.clear();
  }
  size_t AbsorbExtra(const std::vector<uint64_t> &All) override {
    size_t added = 0;
    for (uint64_t v : All) added += aggregate_.insert(v).second;
    return added;
  }
  std::vector<uint64_t> extra_new_;  // aggregate values outside the map since TakeNewExtra
  size_t MergeCoverageMap(const uint8_t *Merged, uint64_t Bytes, bool Device) override {
    if (Device || Bytes != map_.size()) return 0;
    for (uint64_t i = 0; i < Bytes; i++) map_[i] = std::max(map_[i], Merged[i]);
    return AbsorbCoverageMap();
  }
  size_t AbsorbCoverageMap() override {
    size_t added = 0;
    for (size_t i = 0; i < map_.size(); i++)
      if (map_[i] && !shadow_[i]) {
        shadow_[i] = 1;
        added += aggregate_.insert((slot_vpn_[i / 4096] << 12) | (i % 4096)).second;
      }
    return added;
  }
  uint64_t Icount() const { return orc_icount(m_); }
  void RunStats(LaneResult &L) const {
    L.bytes = orc_bytes(m_);
    L.dirty = (uint32_t)orc_dirty(m_, nullptr, 0);
    L.edges = orc_edges(m_, &L.edges_new);
  }
  void PrintRunStats() override {
    LaneResult L;
    L.icount = orc_icount(m_);
    RunStats(L);
    PrintTestcaseRunStats(L, aggregate_.size());
  }
  const ModuleInstances *route_ = nullptr;  // RunBatch over per-lane module copies
  uint32_t route_lane_ = 0;
  bool full_ = false;
  bool engine_error_ = false;
  bool handler_fault_ = false;  // U43 (within engine_error_)
  UnimplHist unimpl_;  // WTF_UNIMPL_HIST=1: printed to stderr at exit
  void SetFullCoverage(bool On) override { full_ = On; }
  size_t CoverageSize() const override { return aggregate_.size(); }
  bool EnableTrace(uint32_t PerLane) override {
    trace_cap_ = PerLane;
    orc_set_trace(m_, PerLane != 0);
    return true;
  }
  bool LaneTrace(uint32_t Lane, std::vector<uint64_t> &Rips, bool &Truncated) override {
    if (Lane >= traces_.size()) return false;
    Rips = traces_[Lane];
    Truncated = Rips.size() > trace_cap_;
    if (Truncated) Rips.resize(trace_cap_);
    return true;
  }
  uint64_t tenet_cap_ = 0;                       // Tenet stream bytes per lane (EnableTenet)
  std::vector<std::vector<uint8_t>> tenets_;     // per testcase of the last RunBatch, untruncated
  bool EnableTenet(uint64_t BytesPerLane) override {
    tenet_cap_ = BytesPerLane;
    orc_set_tenet(m_, BytesPerLane != 0);
    return true;
  }
  bool LaneTenet(uint32_t Lane, std::vector<uint8_t> &Bytes, bool &Truncated) override {
    if (Lane >= tenets_.size()) return false;
    Bytes = tenets_[Lane];
    Truncated = Bytes.size() > tenet_cap_;
    if (Truncated) Bytes.resize(tenet_cap_);
    return true;
  }
  bool RunBatch(const Target_t &Target, const std::vector<std::pair<const uint8_t *, size_t>> &Tc,
                std::vector<LaneResult> &Out, ModuleSlots *Slots) override {
    Out.assign(Tc.size(), LaneResult{});
    route_ = Slots ? Slots->Instances() : nullptr;
    if (trace_cap_) traces_.assign(Tc.size(), {});
    if (tenet_cap_) tenets_.assign(Tc.size(), {});
    g_Backend = this;
    for (size_t i = 0; i < Tc.size(); i++) {
      LaneResult &L = Out[i];
      Restore(initial_);
      route_lane_ = (uint32_t)i;
      const Target_t &T = route_ ? route_->TargetOf((uint32_t)i) : Target;
      bool inserted = false;
      try {
        inserted = T.InsertTestcase(Tc[i].first, Tc[i].second);
      } catch (const HandlerFault_t &) {  // U43
        engine_error_ = true;
        handler_fault_ = true;
      }
      if (!inserted) result_ = Crash_t(engine_error_ ? "" : "insert-testcase-failed");
      std::optional<TestcaseResult_t> R;
      if (result_) {
        R = result_;
        last_new_.clear();
      } else {
        R = Run(Tc[i].first, Tc[i].second);
      }
      L.result = *R;
      L.error = engine_error_;
      L.handler_fault = handler_fault_;
      if (L.error) L.result = Crash_t();
      engine_error_ = false;
      handler_fault_ = false;
      if (std::holds_alternative<Timedout_t>(*R)) {
        L.new_coverage.assign(0, 0);
        for (const Gva_t &g : last_new_) L.new_coverage.push_back(g.U64());
        RevokeLastNewCoverage();
      } else {
        for (const Gva_t &g : last_new_) L.new_coverage.push_back(g.U64());
      }
      const wtfgpu_regs_t r = regs();
      memcpy(L.gprs, r.gpr, 16 * 8);
      L.gprs[16] = r.rip;
      L.gprs[17] = r.rflags;
      L.rip = r.rip;
      L.icount = orc_icount(m_);
      L.bytes = orc_bytes(m_);
      L.dirty = (uint32_t)orc_dirty(m_, nullptr, 0);
      L.edges = orc_edges(m_, &L.edges_new);
      if (trace_cap_) {  // this testcase's rip trace
        std::vector<uint64_t> &T = traces_[i];
        T.resize(orc_trace(m_, nullptr, 0));
        orc_trace(m_, T.data(), T.size());
      }
      if (tenet_cap_) {  // and its Tenet stream
        std::vector<uint64_t> W(orc_tenet(m_, nullptr, 0));
        orc_tenet(m_, W.data(), W.size());
        tenets_[i].assign((const uint8_t *)W.data(), (const uint8_t *)(W.data() + W.size()));
      }
      T.Restore();
    }
    Restore(initial_);
    route_ = nullptr;
    return true;
  }
  std::string StatsJson() const override {
    return "{\"kind\":\"twin\",\"retired\":" + std::to_string(retired_total_) + "}";
  }
};

uint64_t TwinBackend_t::Rdrand() { return wtf_rdrand(seed_); }


int main(int argc, char **argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  RunnerOptions O;
  if (!ParseRunnerArgs(argc, argv, O)) return 2;
  if (O.mode == "master") return MasterMain(O);
  Options_t Opts;
  CpuState_t State;
  if (!LoadTarget(O, Opts, State)) return 1;
  auto *B = new TwinBackend_t();
  g_Backend = B;
  if (!B->Initialize(Opts, State)) return 1;
  // the runner sizes batches by Lanes(); the twin takes the requested lane count
  struct Sized final : Executor_t {
    TwinBackend_t *b;
    uint32_t n;
    Backend_t *AsBackend() override { return b; }
    uint32_t Lanes() const override { return n; }
    bool RunBatch(const Target_t &T, const std::vector<std::pair<const uint8_t *, size_t>> &Tc,
                  std::vector<LaneResult> &Out, ModuleSlots *S) override {
      return b->RunBatch(T, Tc, Out, S);
    }
    void ResetCoverage() override { b->ResetCoverage(); }
    void SetFullCoverage(bool On) override { b->SetFullCoverage(On); }
    size_t CoverageSize() const override { return b->CoverageSize(); }
    std::string StatsJson() const override { return b->StatsJson(); }
    bool CoverageMap(uint8_t **M, uint64_t *N, bool *D) override { return b->CoverageMap(M, N, D); }
    size_t AbsorbCoverageMap() override { return b->AbsorbCoverageMap(); }
    size_t MergeCoverageMap(const uint8_t *M, uint64_t N, bool D) override { return b->MergeCoverageMap(M, N, D); }
    void TakeNewExtra(std::vector<uint64_t> &O) override { b->TakeNewExtra(O); }
    size_t AbsorbExtra(const std::vector<uint64_t> &A) override { return b->AbsorbExtra(A); }
    bool EnableTrace(uint32_t P) override { return b->EnableTrace(P); }
    uint64_t LastIcount() const override { return b->Icount(); }
    bool LastError() const override { return b->engine_error_; }
    bool LastHandlerFault() const override { return b->handler_fault_; }
    void LastRunStats(LaneResult &L) const override { b->RunStats(L); }
    bool LaneTrace(uint32_t L, std::vector<uint64_t> &R, bool &T) override { return b->LaneTrace(L, R, T); }
    bool EnableTenet(uint64_t P) override { return b->EnableTenet(P); }
    bool LaneTenet(uint32_t L, std::vector<uint8_t> &R, bool &T) override { return b->LaneTenet(L, R, T); }
    // WTF_TWIN_STREAM=1: the streaming interface of the gpu node (continuous
    // batching), served synchronously (every lane free at every step, each
    // step's testcases run to their end), so the CPU tests drive the fuzz
    // loop's streaming bookkeeping (runner.cc FuzzSession::StreamStep)
    bool stream = false;
    std::vector<LaneResult> res;  // the last step's results (valid until the next step)
    bool CanStream() const override { return stream; }
    uint32_t FreeLanes() const override { return n; }
    bool StreamStep(const Target_t &T, const std::vector<StreamTestcase_t> &In, uint64_t,
                    std::vector<StreamResult_t> &Out, ModuleSlots *S, size_t *Taken) override {
      const size_t k = std::min<size_t>(In.size(), n);
      if (Taken) *Taken = k;
      std::vector<std::pair<const uint8_t *, size_t>> Tc(k);
      for (size_t i = 0; i < k; i++) Tc[i] = {In[i].data, In[i].size};
      Out.clear();
      if (k == 0) return true;
      if (!b->RunBatch(T, Tc, res, S)) return false;
      for (size_t i = 0; i < k; i++) Out.push_back(StreamResult_t{In[i].tag, &res[i]});
      return true;
    }
  } E;
  E.b = B;
  E.n = O.lanes ? O.lanes : 1;
  E.stream = getenv("WTF_TWIN_STREAM") && getenv("WTF_TWIN_STREAM")[0] == '1';
  // CPU shards merge their host coverage maps over TCP (net_exchange.cc)
  std::unique_ptr<TcpExchange_t> X;
  if (O.world > 1) {
    const size_t colon = O.exchange.rfind(':');
    X = std::make_unique<TcpExchange_t>(O.rank, O.world);
    if (colon == std::string::npos ||
        !X->Connect(O.exchange.substr(0, colon), (uint16_t)atoi(O.exchange.c_str() + colon + 1))) {
      printf("coverage exchange %s failed\n", O.exchange.c_str());
      return 1;
    }
  }
  return RunnerMain(O, E, Opts, State, X.get());
}
