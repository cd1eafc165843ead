// engine_sys.h — system, control-transfer, I/O and x87-control instructions
// of the interpreter (conventions U24-U35; the oracle's
// x86_oracle_sys.inc states the same semantics). One noinline entry,
// sys2_exec, reached from exec() for UOps with op O_SYS2: `sub` holds the
// opcode (0x100 | opcode for the 0f map), asz the operand size, bsz 2 when a
// 66 prefix is present (8 otherwise), imm the immediate (enter: size | level
// << 16).
//
// These are rare instructions, so the code favours few live registers over
// speed. The restart rule of exec() holds: lane state (registers, cold state,
// cpl) changes only after the last access that can miss; instructions that
// write several places first make every page of the written range private
// and writable (span_w), so a copy-on-write restart never repeats a write
// that a later read of the same instruction could observe.
#pragma once
#include "engine_exec.h"

namespace wtfgpu_dev {

constexpr u32 VEC_DB = 1, VEC_NM = 7, VEC_NP = 11, VEC_MF = 16;
constexpr u64 XS_SUPPORTED = 0xff;  // x87, SSE, AVX, BNDREGS, BNDCSR, opmask, ZMM_Hi256, Hi16_ZMM (U33, U47)
// components 2..7: size and standard-format offset (CPUID.(0xd, i)); the
// compacted format packs the requested ones in order (none is 64-byte aligned)
__host__ __device__ constexpr u32 xs_size(u32 c) {
  return c == 2 ? 256 : c == 3 || c == 4 || c == 5 ? 64 : c == 6 ? 512 : c == 7 ? 1024 : 0;
}
__host__ __device__ constexpr u32 xs_offset(u32 c) {
  return c == 2 ? 576 : c == 3 ? 960 : c == 4 ? 1024 : c == 5 ? 1088 : c == 6 ? 1152 : c == 7 ? 1664 : 0;
}

__device__ __forceinline__ u32 lane_iopl(const Lane &L) { return (u32)(L.rflags >> 12) & 3; }


// implicit supervisor access: the walk without permission checks; a
// non-canonical address or a missing page is #PF(err) at va
__device__ __noinline__ bool sup_pa(const Dev &P, Lane &L, u64 va, u32 err, u64 &gpa) {
  u64 td, gpfn;
  const u32 cpl = L.cpl;
  L.cpl = 0;
  const bool ok = canonical(va) && walk(P, L, va, ACC_R, td, gpfn);
  L.cpl = cpl;
  if (!ok) {
    set_fault(L, WTFGPU_VEC_PF, err, va);
    return false;
  }
  gpa = (gpfn << 12) | (va & 0xfff);
  return true;
}
__device__ __forceinline__ bool sup_read_q(const Dev &P, Lane &L, u64 va, u64 &v) {
  u64 ga;
  if (!sup_pa(P, L, va, 0, ga)) return false;
  if ((ga & 0xfff) > 4096 - 8) {
    set_fault(L, WTFGPU_VEC_PF, 0, va);
    return false;
  }
  bool priv;
  const u8 *p = phys_page(P, L.lane, L.ovn, L.bloom, ga >> 12, priv) + (ga & 0xfff);
  u64 x = 0;
  for (int i = 0; i < 8; i++) x |= (u64)p[i] << (8 * i);
  v = x;
  return true;
}
// one aligned qword at gpa into the lane's overlay (copy-on-write + dirty)
__device__ __forceinline__ bool sup_write_pa(const Dev &P, Lane &L, u64 gpa, u64 v) {
  bool priv;
  const u8 *pg = phys_page(P, L.lane, L.ovn, L.bloom, gpa >> 12, priv);
  u8 *dst = (u8 *)pg;
  if (!priv) {
    if (L.ovn >= P.K) {
      L.status = WTFGPU_EXIT_OVERLAY_FULL;
      return false;
    }
    dst = cow_copy(P, L.lane, L.ovn, gpa >> 12, pg);
    L.ovn++;
    L.bloom |= bloom_bit(gpa >> 12);
    L.flush = 1;  // cached translations may point at the shared copy
  }
  *(u64 *)(dst + (gpa & 0xfff)) = v;
  return true;
}

__device__ __forceinline__ int fault_x(Lane &L, u32 vec, u32 err) {
  set_fault(L, vec, err, 0);
  return X_FAULT;
}

// ---------------------------------------------------------------- U24
__device__ __noinline__ int soft_int(const Dev &P, Lane &L, u32 vec, bool dpl_check, u64 nrip, u64 &next) {
  LaneSys &S = P.sys[L.lane];
  const u32 ocpl = L.cpl, ev = vec * 8 + 2;
  if ((u64)vec * 16 + 15 > S.idtr_limit) return fault_x(L, WTFGPU_VEC_GP, ev);
  const u64 ga = P.full[L.lane].idtr_base + (u64)vec * 16;
  u64 g0, g1;
  if (!sup_read_q(P, L, ga, g0) || !sup_read_q(P, L, ga + 8, g1)) return X_FAULT;
  const u32 attr = (u32)(g0 >> 40) & 0xff, type = attr & 0xf, ist = (u32)(g0 >> 32) & 7, dpl = (attr >> 5) & 3;
  if (type != 0xe && type != 0xf) return fault_x(L, WTFGPU_VEC_GP, ev);
  if (dpl_check && dpl < ocpl) return fault_x(L, WTFGPU_VEC_GP, ev);
  if (!(attr & 0x80)) return fault_x(L, VEC_NP, ev);
  const u64 target = (g0 & 0xffff) | ((g0 >> 32) & 0xffff0000ull) | (g1 << 32);
  const u32 sel = (u32)(g0 >> 16) & 0xffff, ncpl = sel & 3;
  if ((sel & 0xfffc) == 0) return fault_x(L, WTFGPU_VEC_GP, 0);
  if (ncpl > ocpl) return fault_x(L, WTFGPU_VEC_GP, sel & 0xfffc);
  if (!canonical(target)) return fault_x(L, WTFGPU_VEC_GP, 0);
  u64 rsp = R(L, 4);
  if (ist || ncpl < ocpl) {
    const u64 off = ist ? 0x24 + (u64)(ist - 1) * 8 : 4 + (u64)ncpl * 8;
    if (!sup_read_q(P, L, S.tss + off, rsp)) return X_FAULT;
  }
  rsp &= ~0xfull;
  // every frame word translates before the first is written
  u64 pa[5];
  for (u32 i = 0; i < 5; i++)
    if (!sup_pa(P, L, rsp - 40 + 8 * i, 2, pa[i])) return X_FAULT;
  const u64 frame[5] = {nrip, S.cs, L.rflags, R(L, 4), S.ss};
  for (u32 i = 0; i < 5; i++)
    if (!sup_write_pa(P, L, pa[i], frame[i])) return X_FAULT;
  if (ncpl < ocpl) S.ss = (u16)ncpl;
  set_cs(L, S, sel);
  if (ncpl != ocpl) L.flush = 1;
  L.cpl = S.cpl = ncpl;
  RS(L, 4, rsp - 40);
  L.rflags &= ~(0x100ull | 0x4000ull | 0x10000ull | 0x20000ull | (type == 0xe ? 0x200ull : 0));
  next = target;
  return X_OK;
}

// ---------------------------------------------------------------- U27
// CPUID: the fixed table (the oracle's cpuid_leaf states the same values)
__device__ __noinline__ void cpuid_leaf(u64 cr4, u64 xcr0, u32 leaf, u32 sub, u32 *r) {
  r[0] = r[1] = r[2] = r[3] = 0;
  const u32 osxsave = (u32)(cr4 >> 18) & 1;
  if (leaf == 0) {
    r[0] = 0xd;
    r[1] = 0x756e6547;
    r[3] = 0x49656e69;
    r[2] = 0x6c65746e;
  } else if (leaf == 1) {
    r[0] = 0x000906ea;
    r[1] = 0x00000800;
    // SSE3, PCLMULQDQ, SSSE3, FMA, CX16, SSE4.1, SSE4.2, MOVBE, POPCNT, AES, XSAVE, OSXSAVE, AVX, F16C, RDRAND
    r[2] = (1u << 0) | (1u << 1) | (1u << 9) | (1u << 12) | (1u << 13) | (1u << 19) | (1u << 20) | (1u << 22) |
           (1u << 23) | (1u << 25) | (1u << 26) | (osxsave << 27) | (1u << 28) | (1u << 29) | (1u << 30);
    r[3] = 0x078bfbfd;
  } else if (leaf == 7) {
    if (sub == 0) {  // FSGSBASE BMI1 AVX2 BMI2 ERMS RTM AVX512F ADX SHA AVX512BW AVX512VL (U47, U48)
      r[1] = (1u << 0) | (1u << 3) | (1u << 5) | (1u << 8) | (1u << 9) | (1u << 11) | (1u << 16) | (1u << 19) |
             (1u << 29) | (1u << 30) | (1u << 31);
      r[3] = 1u << 11;  // RTM_ALWAYS_ABORT: xbegin always aborts (U48)
    }
  } else if (leaf == 0xd) {
    if (sub == 0) {
      r[0] = 0xff;
      r[1] = 576;
      for (u32 c = 2; c <= 7; c++)
        if ((xcr0 >> c) & 1) r[1] = xs_offset(c) + xs_size(c);
      r[2] = 2688;
    } else if (sub == 1) {
      r[0] = 1u | 2u | 8u;
      r[1] = 576;
      for (u32 c = 2; c <= 7; c++)
        if ((xcr0 >> c) & 1) r[1] += xs_size(c);
    } else if (sub >= 2 && sub <= 7) {
      r[0] = xs_size(sub);
      r[1] = xs_offset(sub);
    }
  } else if (leaf == 0x80000000u) {
    r[0] = 0x80000008u;
  } else if (leaf == 0x80000001u) {
    r[2] = (1u << 0) | (1u << 5) | (1u << 8);
    r[3] = (1u << 11) | (1u << 20) | (1u << 26) | (1u << 27) | (1u << 29);
  } else if (leaf >= 0x80000002u && leaf <= 0x80000004u) {
    // "wtf gpu backend x86-64 interpreter (MI355X)     "
    const char brand[49] = "wtf gpu backend x86-64 interpreter (MI355X)     ";
    const u32 base = 16 * (leaf - 0x80000002u);
    for (u32 i = 0; i < 16; i++) r[i >> 2] |= (u32)(u8)brand[base + i] << (8 * (i & 3));
  } else if (leaf == 0x80000008u) {
    r[0] = 0x3030;
  }
}

// ---------------------------------------------------------------- U30
// sreg: 0 es 2 ss 3 ds 4 fs 5 gs (cs never loaded here). true = loaded.
__device__ __noinline__ bool load_sreg(const Dev &P, Lane &L, u32 sreg, u32 sel, bool commit) {
  wtfgpu_regs_t &F = P.full[L.lane];
  if (sreg == WTFGPU_SS && (sel & 0xfffc) == 0 && L.cpl == 3) {
    set_fault(L, WTFGPU_VEC_GP, 0, 0);
    return false;
  }
  u64 base = 0;
  const bool fsgs = (sreg == WTFGPU_FS || sreg == WTFGPU_GS) && (sel & 0xfffc);
  if (fsgs) {
    if ((sel & 4) || (u64)(sel | 7) > F.gdtr_limit) {
      set_fault(L, WTFGPU_VEC_GP, sel & 0xfffc, 0);
      return false;
    }
    u64 dsc;
    if (!sup_read_q(P, L, F.gdtr_base + (sel & 0xfff8), dsc)) return false;
    if (!((dsc >> 47) & 1)) {
      set_fault(L, VEC_NP, sel & 0xfffc, 0);
      return false;
    }
    base = ((dsc >> 16) & 0xffffff) | (((dsc >> 56) & 0xff) << 24);
  }
  if (!commit) return true;
  if (fsgs) {
    if (sreg == WTFGPU_FS) P.fs_base[L.lane] = base;
    else P.gs_base[L.lane] = base;
  }
  if (sreg == WTFGPU_SS) P.sys[L.lane].ss = (u16)sel;
  else F.seg[sreg].selector = (u16)sel;
  return true;
}

// GDT descriptor of a selector (LAR / LSL / VERR / VERW): 0 found, 1 not
// usable (ZF := 0), -1 fault
__device__ __forceinline__ int gdt_desc(const Dev &P, Lane &L, u32 sel, u64 &dsc) {
  const wtfgpu_regs_t &F = P.full[L.lane];
  if ((sel & 0xfffc) == 0 || (sel & 4) || (u64)(sel | 7) > F.gdtr_limit) return 1;
  return sup_read_q(P, L, F.gdtr_base + (sel & 0xfff8), dsc) ? 0 : -1;
}

// ---------------------------------------------------------------- U32 / U33
__device__ __forceinline__ u32 ftw_abridged(u32 ftw) {
  u32 t = 0;
  for (int i = 0; i < 8; i++)
    if (((ftw >> (2 * i)) & 3) != 3) t |= 1u << i;
  return t;
}
__device__ __forceinline__ u32 tag_of(u64 mant, u32 se) {
  const u32 e = se & 0x7fff;
  if (e == 0x7fff) return 2;
  if (e == 0) return mant ? 2 : 1;
  return (mant >> 63) ? 0 : 2;
}
// FSW after loading a status / control pair: ES and B follow the unmasked
// flags (what the host's FXRSTOR / FRSTOR / FLDENV do, U42)
__device__ __forceinline__ u32 fsw_norm(u32 fsw, u32 fcw) {
  return (fsw & 0x7f7fu) | ((fsw & ~fcw & 0x3fu) ? 0x8080u : 0u);
}
// a waiting x87 instruction takes #MF while an unmasked exception flag is set
__device__ __forceinline__ bool x87_pending(const wtfgpu_regs_t &F) { return (F.fpsw & ~F.fpcw & 0x3f) != 0; }
__device__ __forceinline__ u32 mxcsr_mask_of(const wtfgpu_regs_t &F) { return F.mxcsr_mask ? F.mxcsr_mask : 0xffbfu; }

// 8 bytes of the legacy (FXSAVE) image at offset off (a multiple of 8, < 416)
__device__ __noinline__ u64 legacy_q(const Dev &P, const Lane &L, u32 off) {
  const wtfgpu_regs_t &F = P.full[L.lane];
  if (off == 0)
    return (u64)F.fpcw | ((u64)F.fpsw << 16) | ((u64)ftw_abridged(F.fptw) << 32) | ((u64)F.fpop << 48);
  if (off < 24) return 0;
  if (off == 24) return (u64)F.mxcsr | ((u64)mxcsr_mask_of(F) << 32);
  if (off < 160) {
    const u32 k = (off - 32) >> 4;
    return (off & 8) ? (u64)F.fpse[k] : F.fpst[k];
  }
  const u32 k = (off - 160) >> 4;
  return F.xmm[k][(off >> 3) & 1];
}

__device__ __forceinline__ void x87_init(wtfgpu_regs_t &F) {
  F.fpcw = 0x37f;
  F.fpsw = 0;
  F.fptw = 0xffff;
  F.fpop = 0;
  for (int i = 0; i < 8; i++) F.fpst[i] = 0, F.fpse[i] = 0;
}

// FNINIT: control / status / tags reset, TOP = 0 (ST order rotated to R order),
// the register contents kept
__device__ __forceinline__ void x87_fninit(wtfgpu_regs_t &F) {
  const u32 top = (F.fpsw >> 11) & 7;
  u64 t[8];
  u16 e[8];
  for (u32 j = 0; j < 8; j++) t[j] = F.fpst[(j - top) & 7], e[j] = F.fpse[(j - top) & 7];
  for (u32 j = 0; j < 8; j++) F.fpst[j] = t[j], F.fpse[j] = e[j];
  F.fpcw = 0x37f;
  F.fpsw = 0;
  F.fptw = 0xffff;
  F.fpop = 0;
}

// bytes [off, off + n) of the legacy region written with vwrite (n a multiple of 8)
__device__ __noinline__ bool legacy_store(const Dev &P, Lane &L, u64 va, u32 off, u32 n) {
  for (u32 o = off; o < off + n; o += 8)
    if (!vwrite(L, va + o, 8, legacy_q(P, L, o))) return false;
  return true;
}

// the x87 part of an FXRSTOR / XRSTOR image: first 8 bytes (fcw fsw ftw fop),
// then ST0..7 (8 significand bytes and the sign / exponent word each)
__device__ __noinline__ bool x87_load(const Dev &P, Lane &L, u64 va, bool commit) {
  u64 q0;
  if (!vread(L, va, 8, q0)) return false;
  u64 mant[8];
  u32 se[8];
  for (u32 i = 0; i < 8; i++) {
    u64 s2;
    if (!vread(L, va + 32 + 16 * i, 8, mant[i]) || !vread(L, va + 40 + 16 * i, 8, s2)) return false;
    se[i] = (u32)s2 & 0xffff;
  }
  if (!commit) return true;
  wtfgpu_regs_t &F = P.full[L.lane];
  const u32 fsw = (u32)(q0 >> 16) & 0xffff, abr = (u32)(q0 >> 32) & 0xff, top = (fsw >> 11) & 7;
  u32 w = 0;
  for (u32 p = 0; p < 8; p++) {
    u32 t = 3;
    if ((abr >> p) & 1) {
      const u32 s = (p - top) & 7;
      t = tag_of(mant[s], se[s]);
    }
    w |= t << (2 * p);
  }
  F.fpcw = (u16)q0;
  F.fpsw = (u16)fsw_norm(fsw, (u32)q0 & 0xffff);
  F.fptw = (u16)w;
  F.fpop = (u16)((q0 >> 48) & 0x7ff);
  for (u32 i = 0; i < 8; i++) F.fpst[i] = mant[i], F.fpse[i] = (u16)se[i];
  return true;
}

enum : u32 { XS_SAVE, XS_SAVEOPT, XS_SAVEC, XS_SAVES, XS_RSTOR, XS_RSTORS };
__device__ __forceinline__ u32 xs_extent(u64 rfbm, bool compact) {
  u32 n = 576;
  for (u32 c = 2; c <= 7; c++)
    if ((rfbm >> c) & 1) n = compact ? n + xs_size(c) : xs_offset(c) + xs_size(c);
  return n;
}
// the AVX-512 components' 8-byte words: 5 = k0..k7, 6 = zmm0..15 bits
// 511:256, 7 = zmm16..31
__device__ __forceinline__ u64 &xs_word(wtfgpu_regs_t &F, u32 c, u32 i) {
  return c == 5 ? F.k[i] : c == 6 ? F.zmmh[i >> 2][i & 3] : F.zmm_hi[i >> 3][i & 7];
}

__device__ __noinline__ int xsave_op(const Dev &P, Lane &L, u32 kind, u64 va) {
  const LaneSys &S = P.sys[L.lane];
  wtfgpu_regs_t &F = P.full[L.lane];
  if (!((S.cr4 >> 18) & 1)) return fault_x(L, WTFGPU_VEC_UD, 0);
  if (L.cr0 & 8) return fault_x(L, VEC_NM, 0);
  if ((kind == XS_SAVES || kind == XS_RSTORS) && L.cpl != 0) return fault_x(L, WTFGPU_VEC_GP, 0);
  if (va & 63) return fault_x(L, WTFGPU_VEC_GP, 0);
  const u64 rfbm = F.xcr0 & XS_SUPPORTED & ((R(L, 2) << 32) | (R(L, 0) & 0xffffffffull));
  if (kind <= XS_SAVES) {
    const bool compact = kind == XS_SAVEC || kind == XS_SAVES;
    if (!span_w(L, va, xs_extent(rfbm, compact))) return X_FAULT;
    u64 bv = 0;
    if (!compact && !vread(L, va + 512, 8, bv)) return X_FAULT;
    const u64 inuse = rfbm & 0xe7;
    if ((rfbm & 1) && (!legacy_store(P, L, va, 0, 24) || !legacy_store(P, L, va, 32, 128))) return X_FAULT;
    // MXCSR / MXCSR_MASK: with SSE or AVX requested, but compacted only with SSE (native images)
    if ((rfbm & (compact ? 2 : 6)) && !legacy_store(P, L, va, 24, 8)) return X_FAULT;
    if ((rfbm & 2) && !legacy_store(P, L, va, 160, 256)) return X_FAULT;
    if (compact) {
      if (!vwrite(L, va + 512, 8, inuse) || !vwrite(L, va + 520, 8, 0x8000000000000000ull | rfbm)) return X_FAULT;
    } else {
      if (!vwrite(L, va + 512, 8, (bv & ~rfbm) | inuse)) return X_FAULT;
    }
    u32 off = 576;
    if (rfbm & 4) {
      for (u32 i = 0; i < 32; i++)
        if (!vwrite(L, va + off + 8 * i, 8, F.ymmh[i >> 1][i & 1])) return X_FAULT;
      off += 256;
    }
    for (u32 c = 3; c <= 7; c++)
      if ((rfbm >> c) & 1) {
        const u64 at = compact ? off : xs_offset(c);
        for (u32 i = 0; i < xs_size(c) / 8; i++)
          if (!vwrite(L, va + at + 8 * i, 8, c >= 5 ? xs_word(F, c, i) : 0)) return X_FAULT;
        off += xs_size(c);
      }
    return X_OK;
  }
  // XRSTOR / XRSTORS: the header, then every check, then the state
  u64 xbv, xcomp, rest = 0;
  if (!vread(L, va + 512, 8, xbv) || !vread(L, va + 520, 8, xcomp)) return X_FAULT;
  for (u32 i = 2; i < 8; i++) {
    u64 h;
    if (!vread(L, va + 512 + 8 * i, 8, h)) return X_FAULT;
    rest |= h;
  }
  const bool compact = (xcomp >> 63) & 1;
  bool bad = rest != 0 || (kind == XS_RSTORS && !compact);
  if (compact) bad = bad || (xcomp & ~(0x8000000000000000ull | F.xcr0)) || (xbv & ~xcomp & ~0x8000000000000000ull);
  else bad = bad || xcomp != 0 || (xbv & ~F.xcr0);
  if (bad) return fault_x(L, WTFGPU_VEC_GP, 0);
  // the legacy region is read whole (512 bytes), as the oracle does
  u64 mx = 0;
  for (u32 o = 0; o < 512; o += 8) {
    u64 q;
    if (!vread(L, va + o, 8, q)) return X_FAULT;
    if (o == 24) mx = q & 0xffffffffull;
  }
  const bool load_mx = compact ? ((rfbm & 2) && (xbv & 2)) : ((rfbm & 6) != 0);
  if (load_mx && (mx & ~(u64)mxcsr_mask_of(F))) return fault_x(L, WTFGPU_VEC_GP, 0);
  {  // the extended components read before any commit (compacted: packed in order)
    u32 off = 576;
    for (u32 c = 2; c <= 7; c++) {
      if (compact && !((xcomp >> c) & 1)) continue;
      const u32 at = compact ? off : xs_offset(c);
      off += xs_size(c);
      if (c == 3 || c == 4 || !((rfbm >> c) & 1) || !((xbv >> c) & 1)) continue;
      for (u32 o = 0; o < xs_size(c); o += 8) {
        u64 q;
        if (!vread(L, va + at + o, 8, q)) return X_FAULT;
      }
    }
  }
  // commit: every byte above was read without a miss, so the reads below hit
  // the TLB; they are not counted again (the oracle reads the area once)
  const u32 pend0 = L.pend;
  if (rfbm & 1) {
    if (xbv & 1) x87_load(P, L, va, true);
    else x87_init(F);
  }
  if (rfbm & 2) {
    for (u32 i = 0; i < 16; i++) {
      u64 lo = 0, hi = 0;
      if (xbv & 2) {
        vread(L, va + 160 + 16 * i, 8, lo);
        vread(L, va + 168 + 16 * i, 8, hi);
      }
      F.xmm[i][0] = lo;
      F.xmm[i][1] = hi;
    }
  }
  if (load_mx) F.mxcsr = (u32)mx;
  else if (compact && (rfbm & 2) && !(xbv & 2)) F.mxcsr = 0x1f80;
  {
    u32 off = 576;
    for (u32 c = 2; c <= 7; c++) {
      if (compact && !((xcomp >> c) & 1)) continue;
      const u32 at = compact ? off : xs_offset(c);
      off += xs_size(c);
      if (c == 3 || c == 4 || !((rfbm >> c) & 1)) continue;
      for (u32 i = 0; i < xs_size(c) / 8; i++) {
        u64 q = 0;  // a component not in XSTATE_BV: its initial state (zeros)
        if ((xbv >> c) & 1) vread(L, va + at + 8 * i, 8, q);
        if (c == 2) F.ymmh[i >> 1][i & 1] = q;
        else xs_word(F, c, i) = q;
      }
    }
  }
  L.pend = pend0;
  return X_OK;
}

__device__ __noinline__ int fxsave_op(const Dev &P, Lane &L, bool restore, u64 va) {
  wtfgpu_regs_t &F = P.full[L.lane];
  if (L.cr0 & 0xc) return fault_x(L, VEC_NM, 0);
  if (va & 15) return fault_x(L, WTFGPU_VEC_GP, 0);
  if (!restore) {
    if (!span_w(L, va, 416)) return X_FAULT;
    return legacy_store(P, L, va, 0, 416) ? X_OK : X_FAULT;
  }
  u64 mx = 0;
  for (u32 o = 0; o < 416; o += 8) {
    u64 q;
    if (!vread(L, va + o, 8, q)) return X_FAULT;
    if (o == 24) mx = q & 0xffffffffull;
  }
  if (mx & ~(u64)mxcsr_mask_of(F)) return fault_x(L, WTFGPU_VEC_GP, 0);
  const u32 pend0 = L.pend;  // the re-reads below hit and are not counted again
  x87_load(P, L, va, true);
  F.mxcsr = (u32)mx;
  for (u32 i = 0; i < 16; i++) {
    u64 lo, hi;
    vread(L, va + 160 + 16 * i, 8, lo);
    vread(L, va + 168 + 16 * i, 8, hi);
    F.xmm[i][0] = lo;
    F.xmm[i][1] = hi;
  }
  L.pend = pend0;
  return X_OK;
}

// the 28-byte environment, 8 bytes at off (0, 8, 16; 24 holds 4)
__device__ __forceinline__ u64 env_q(const wtfgpu_regs_t &F, u32 off) {
  if (off == 0) return (u64)F.fpcw | ((u64)F.fpsw << 32);
  if (off == 8) return (u64)F.fptw;
  if (off == 16) return (u64)(F.fpop & 0x7ff) << 16;
  return 0;
}

}  // namespace wtfgpu_dev
#include "engine_x87.h"
namespace wtfgpu_dev {

__device__ __noinline__ int exec_x87(const Dev &P, Lane &L, const UOp &u, u64 va) {
  wtfgpu_regs_t &F = P.full[L.lane];
  const u32 op = u.sub & 0xff, r3 = u.reg & 7, mem = u.is_mem;
  const u32 modrm = 0xc0 | (r3 << 3) | (u.rm & 7);
  bool ctl = false;
  if (op == 0xd9 && mem && r3 >= 4) ctl = true;
  if (op == 0xdb && !mem && (modrm == 0xe2 || modrm == 0xe3)) ctl = true;
  if (op == 0xdd && mem && (r3 == 4 || r3 == 6 || r3 == 7)) ctl = true;
  if (op == 0xdf && !mem && modrm == 0xe0) ctl = true;
  if (!ctl) return x87_arith(P, L, u, va);
  if (mem && (r3 == 4 || r3 == 6) && u.bsz == 2) return X_UNIMPL;  // 16-bit environment formats
  if (L.cr0 & 0xc) return fault_x(L, VEC_NM, 0);
  if (op == 0xdb) {
    if (modrm == 0xe3) x87_fninit(F);
    else F.fpsw &= 0x7f00;
    return X_OK;
  }
  if (op == 0xdf) {
    RS(L, 0, (R(L, 0) & ~0xffffull) | F.fpsw);
    return X_OK;
  }
  if (op == 0xd9) {
    if (r3 == 4) {  // fldenv
      u64 q0, q1, q2, q3;
      if (!vread(L, va, 8, q0) || !vread(L, va + 8, 8, q1) || !vread(L, va + 16, 8, q2) || !vread(L, va + 24, 4, q3))
        return X_FAULT;
      // FCW as FLDCW loads it; the physical registers stay where they are
      // under the loaded TOP (fpst is kept in ST order: rotated as FNINIT
      // does); every tag not empty recomputed from the register's contents
      // (what the host's FNSTENV shows afterwards)
      const u32 ot = (F.fpsw >> 11) & 7, nt = (u32)(q0 >> 43) & 7;
      u64 t[8];
      u16 e[8];
      for (u32 j = 0; j < 8; j++) t[j] = F.fpst[(nt + j - ot) & 7], e[j] = F.fpse[(nt + j - ot) & 7];
      for (u32 j = 0; j < 8; j++) F.fpst[j] = t[j], F.fpse[j] = e[j];
      F.fpcw = (u16)((q0 & ~0xe0c0ull) | 0x40);
      F.fpsw = (u16)fsw_norm((u32)(q0 >> 32) & 0xffff, F.fpcw);
      F.fptw = (u16)q1;
      F.fpop = (u16)((q2 >> 16) & 0x7ff);
      x87_retag(F);
      return X_OK;
    }
    if (r3 == 5) {  // fldcw
      u64 v;
      if (!vread(L, va, 2, v)) return X_FAULT;
      F.fpcw = (u16)((v & ~0xe0c0ull) | 0x40);
      if (F.fpsw & ~F.fpcw & 0x3f) F.fpsw |= 0x8080;
      else F.fpsw &= (u16)~0x8080;
      return X_OK;
    }
    if (r3 == 6) {  // fnstenv, then every exception masked
      if (!span_w(L, va, 28)) return X_FAULT;
      if (!vwrite(L, va, 8, env_q(F, 0)) || !vwrite(L, va + 8, 8, env_q(F, 8)) || !vwrite(L, va + 16, 8, env_q(F, 16)) ||
          !vwrite(L, va + 24, 4, 0))
        return X_FAULT;
      F.fpcw |= 0x3f;
      return X_OK;
    }
    return vwrite(L, va, 2, F.fpcw) ? X_OK : X_FAULT;  // fnstcw
  }
  // dd
  if (r3 == 4) {  // frstor: the environment, then 8 ten-byte registers
    u64 q0, q1, q2, q3;
    if (!vread(L, va, 8, q0) || !vread(L, va + 8, 8, q1) || !vread(L, va + 16, 8, q2) || !vread(L, va + 24, 4, q3))
      return X_FAULT;
    u64 st[8], se[8];
    for (u32 i = 0; i < 8; i++)
      if (!vread(L, va + 28 + 10 * i, 8, st[i]) || !vread(L, va + 36 + 10 * i, 2, se[i])) return X_FAULT;
    F.fpcw = (u16)((q0 & ~0xe0c0ull) | 0x40);
    F.fpsw = (u16)fsw_norm((u32)(q0 >> 32) & 0xffff, F.fpcw);
    F.fptw = (u16)q1;
    F.fpop = (u16)((q2 >> 16) & 0x7ff);
    for (u32 i = 0; i < 8; i++) F.fpst[i] = st[i], F.fpse[i] = (u16)se[i];
    x87_retag(F);
    return X_OK;
  }
  if (r3 == 6) {  // fnsave, then fninit
    if (!span_w(L, va, 108)) return X_FAULT;
    if (!vwrite(L, va, 8, env_q(F, 0)) || !vwrite(L, va + 8, 8, env_q(F, 8)) || !vwrite(L, va + 16, 8, env_q(F, 16)) ||
        !vwrite(L, va + 24, 4, 0))
      return X_FAULT;
    for (u32 i = 0; i < 8; i++)
      if (!vwrite(L, va + 28 + 10 * i, 8, F.fpst[i]) || !vwrite(L, va + 36 + 10 * i, 2, F.fpse[i])) return X_FAULT;
    x87_fninit(F);
    return X_OK;
  }
  return vwrite(L, va, 2, F.fpsw) ? X_OK : X_FAULT;  // fnstsw m16
}

// ---------------------------------------------------------------- U29 far transfers
// far ret (iret = false, imm = the released bytes) / iret with osz-byte slots
// (from 32-bit code, m32: esp addresses the frame, and an iret at the same
// privilege pops no SS:ESP, SDM IRET "IA-32e mode")
__device__ __noinline__ int far_pop(const Dev &P, Lane &L, u32 osz, u64 imm, bool iret, bool m32, u64 &next) {
  LaneSys &S = P.sys[L.lane];
  const u64 smask = m32 ? 0xffffffffull : ~0ull;
  const u64 rsp = R(L, 4) & smask;
  const u32 ocpl = L.cpl;
  u64 f0, f1, f2 = 0, f3 = 0, f4 = 0;
  if (!vread(L, rsp, osz, f0) || !vread(L, (rsp + osz) & smask, osz, f1)) return X_FAULT;
  if (iret && !vread(L, (rsp + 2 * osz) & smask, osz, f2)) return X_FAULT;
  const u32 cs = (u32)f1 & 0xffff, ncpl = cs & 3;
  const bool outer = iret ? (!m32 || ncpl > ocpl) : ncpl > ocpl;  // SS:RSP popped
  if (iret && outer && (!vread(L, (rsp + 3 * osz) & smask, osz, f3) || !vread(L, (rsp + 4 * osz) & smask, osz, f4)))
    return X_FAULT;
  if ((cs & 0xfffc) == 0 || ncpl < ocpl) return fault_x(L, WTFGPU_VEC_GP, cs & 0xfffc);
  u64 nrsp = (rsp + (iret ? 3 : 2) * (u64)osz + imm) & smask, nss = S.ss;
  if (!iret && ncpl > ocpl) {
    if (!vread(L, (rsp + 2 * (u64)osz + imm) & smask, osz, f3) || !vread(L, (rsp + 3 * (u64)osz + imm) & smask, osz, f4))
      return X_FAULT;
  }
  if (outer) {
    nss = f4 & 0xffff;
    nrsp = f3 + (iret ? 0 : imm);
    if ((nss & 0xfffc) == 0 && ncpl == 3) return fault_x(L, WTFGPU_VEC_GP, 0);
  }
  if (!canonical(f0)) return fault_x(L, WTFGPU_VEC_GP, 0);
  // to SYSRET's compatibility-mode selector (U29): a rip past the 32-bit
  // segment's limit is #GP(0)
  const bool compat = compat_sel(S.star, cs);
  if (compat && (f0 >> 32)) return fault_x(L, WTFGPU_VEC_GP, 0);
  if (iret) {
    u64 mask = 0x254dd5ull;
    if (ocpl == 0) mask |= 0x200ull | 0x3000ull | 0x80000ull | 0x100000ull;
    else if (ocpl <= lane_iopl(L)) mask |= 0x200ull;
    if (osz == 2) mask &= 0xffff;
    L.rflags = (L.rflags & ~mask) | (f2 & mask) | 2;
  }
  set_cs(L, S, cs);
  S.ss = (u16)nss;
  if (ncpl != ocpl) L.flush = 1;
  L.cpl = S.cpl = ncpl;
  RS(L, 4, nrsp);
  next = f0;
  return X_OK;
}

// ---------------------------------------------------------------- 32-bit code (U29)
// The one-byte forms 64-bit mode leaves #UD: push / pop es cs ss ds, pusha /
// popa, the BCD adjustments, far call / jmp ptr16:32, into. BCD flags the SDM
// leaves undefined follow a logical result (SF ZF PF of AL, OF 0; U29).
__device__ __noinline__ int sys32_exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next) {
  LaneSys &S = P.sys[L.lane];
  wtfgpu_regs_t &F = P.full[L.lane];
  const u32 c = u.sub & 0xff, osz = u.asz, sl = u.bsz;  // operand size, stack slot
  const u64 esp = R(L, 4) & 0xffffffffull;
  const u64 al = R(L, 0) & 0xff, ah = (R(L, 0) >> 8) & 0xff;
  auto set_al_flags = [&](u64 nal, u64 nah, u64 cf, u64 af) {
    RS(L, 0, (R(L, 0) & ~0xffffull) | (nah << 8) | (nal & 0xff));
    L.rflags = (L.rflags & ~F_STATUS) | szp(nal & 0xff, 1) | (cf ? F_CF : 0) | (af ? F_AF : 0);
  };
  switch (c) {
    case 0x06: case 0x0e: case 0x16: case 0x1e: {  // push es / cs / ss / ds
      const u32 r = c >> 3;
      const u64 v = r == WTFGPU_CS ? S.cs : r == WTFGPU_SS ? S.ss : F.seg[r].selector;
      if (!vwrite(L, (esp - sl) & 0xffffffffull, sl, v)) return X_FAULT;
      RS(L, 4, (esp - sl) & 0xffffffffull);
      return X_OK;
    }
    case 0x07: case 0x17: case 0x1f: {  // pop es / ss / ds
      u64 v;
      if (!vread(L, esp, sl, v)) return X_FAULT;
      if (!load_sreg(P, L, c >> 3, (u32)v & 0xffff, true)) return X_FAULT;
      RS(L, 4, (esp + sl) & 0xffffffffull);
      return X_OK;
    }
    case 0x60: {  // pusha: eax ecx edx ebx esp(before) ebp esi edi, eax highest
      if (!span_w(L, (esp - 8 * osz) & 0xffffffffull, 8 * osz)) return X_FAULT;
      for (u32 i = 0; i < 8; i++)
        if (!vwrite(L, (esp - (i + 1) * osz) & 0xffffffffull, osz, i == 4 ? esp : R(L, i))) return X_FAULT;
      RS(L, 4, (esp - 8 * osz) & 0xffffffffull);
      return X_OK;
    }
    case 0x61: {  // popa: every slot read before a register changes; esp's slot skipped
      u64 v[8];
      for (u32 i = 0; i < 8; i++)
        if (i != 3 && !vread(L, (esp + i * osz) & 0xffffffffull, osz, v[i])) return X_FAULT;
      for (u32 i = 0; i < 8; i++)
        if (i != 3) setr(L, 0, 7 - i, osz, v[i]);
      RS(L, 4, (esp + 8 * osz) & 0xffffffffull);
      return X_OK;
    }
    case 0x27: case 0x2f: {  // daa / das (bochs' order: CF of the low adjust, then the high)
      const bool cf = L.rflags & F_CF, af = L.rflags & F_AF, sub = c == 0x2f;
      u64 nal = al, ncf = 0, naf = 0;
      if ((al & 0xf) > 9 || af) {
        ncf = cf || (sub ? al < 6 : al > 0xf9);
        nal = (sub ? nal - 6 : nal + 6) & 0xff;
        naf = 1;
      }
      if (al > 0x99 || cf) {
        nal = (sub ? nal - 0x60 : nal + 0x60) & 0xff;
        ncf = 1;
      }
      set_al_flags(nal, ah, ncf, naf);
      return X_OK;
    }
    case 0x37: case 0x3f: {  // aaa / aas
      const bool adj = (al & 0xf) > 9 || (L.rflags & F_AF);
      u64 ax = R(L, 0) & 0xffff;
      if (adj && c == 0x37) ax = ax + 0x106;  // SDM: AX + 106H
      if (adj && c == 0x3f) {                  // SDM: AX - 6, then AH - 1
        ax = (ax - 6) & 0xffff;
        ax = (ax & 0xff) | ((((ax >> 8) - 1) & 0xff) << 8);
      }
      set_al_flags(ax & 0x0f, (ax >> 8) & 0xff, adj, adj);
      return X_OK;
    }
    case 0xd4: {  // aam imm8
      const u64 b = u.imm & 0xff;
      if (b == 0) return fault_x(L, WTFGPU_VEC_DE, 0);
      set_al_flags(al % b, al / b, 0, 0);
      return X_OK;
    }
    case 0xd5:  // aad imm8
      set_al_flags((al + ah * (u.imm & 0xff)) & 0xff, 0, 0, 0);
      return X_OK;
    case 0xce:  // into
      if (!(L.rflags & F_OF)) return X_OK;
      return soft_int(P, L, 4, true, nrip, next);
    case 0x9a: case 0xea: {  // far call / jmp ptr16:32 (ptr16:16 with 66)
      const u64 off = u.imm & (osz == 2 ? 0xffffull : 0xffffffffull), sel = (u.imm >> (8 * osz)) & 0xffff;
      if ((sel & 0xfffc) == 0) return fault_x(L, WTFGPU_VEC_GP, 0);
      if (c == 0x9a) {
        if (!span_w(L, (esp - 2 * osz) & 0xffffffffull, 2 * osz)) return X_FAULT;
        if (!vwrite(L, (esp - osz) & 0xffffffffull, osz, S.cs) || !vwrite(L, (esp - 2 * osz) & 0xffffffffull, osz, nrip))
          return X_FAULT;
        RS(L, 4, (esp - 2 * osz) & 0xffffffffull);
      }
      set_cs(L, S, (u32)((sel & 0xfffc) | L.cpl));
      next = off;
      return X_OK;
    }
    default:
      return X_UNIMPL;
  }
}

// ---------------------------------------------------------------- dispatch
__device__ __noinline__ int sys2_exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next, u64 ea) {
  LaneSys &S = P.sys[L.lane];
  wtfgpu_regs_t &F = P.full[L.lane];
  const u32 c = u.sub & 0xff, map0f = u.sub >> 8, r3 = u.reg & 7, osz = u.asz;
  const bool p66 = u.bsz == 2, rexw = (u.rex >> 3) & 1;
  const bool m32 = u.p67 & 2;  // 32-bit code (U29)
  const u64 smask = m32 ? 0xffffffffull : ~0ull;
  const u32 cpl = L.cpl;
  if (!map0f && m32 && (c < 0x40 || c == 0x60 || c == 0x61 || c == 0x9a || c == 0xce || c == 0xd4 || c == 0xd5 || c == 0xea))
    return sys32_exec(P, L, u, nrip, next);
  const bool umip = (S.cr4 >> 11) & 1;
  u64 a = 0;
  if (!map0f) {
    switch (c) {
      case 0x6c: case 0x6d: case 0x6e: case 0x6f:
        return X_UNIMPL;  // ins / outs run in string_op
      case 0xe4: case 0xe5: case 0xec: case 0xed:  // in: all ones (U31)
        if (cpl > lane_iopl(L)) return fault_x(L, WTFGPU_VEC_GP, 0);
        setr(L, u.rex, 0, (c & 1) ? (osz == 2 ? 2 : 4) : 1, ~0ull);
        return X_OK;
      // 32-bit code only (decode routes them here in compatibility mode, U29)
      case 0x62: {  // bound r, m16&16 / m32&32: #BR unless lower <= index <= upper (signed)
        if (!u.is_mem) return fault_x(L, WTFGPU_VEC_UD, 0);
        u64 lo, hi;
        if (!vread(L, ea, osz, lo) || !vread(L, ea + osz, osz, hi)) return X_FAULT;
        const i64 ix = (i64)sext(R(L, u.reg) & szmask(osz), osz);
        if (ix < (i64)sext(lo, osz) || ix > (i64)sext(hi, osz)) return fault_x(L, 5, 0);
        return X_OK;
      }
      case 0x63: {  // arpl r/m16, r16: the destination selector's RPL raised to the source's (ZF = 1), else ZF = 0
        u64 d;
        if (u.is_mem) {
          if (!vread(L, ea, 2, d, ACC_W)) return X_FAULT;
        } else {
          d = R(L, u.rm) & 0xffff;
        }
        const u64 rpl = R(L, u.reg) & 3;
        const bool adj = (d & 3) < rpl;
        if (adj) {
          d = (d & ~3ull) | rpl;
          if (u.is_mem) {
            if (!vwrite(L, ea, 2, d)) return X_FAULT;
          } else {
            setr(L, 0, u.rm, 2, d);
          }
        }
        L.rflags = (L.rflags & ~F_ZF) | (adj ? F_ZF : 0);
        return X_OK;
      }
      case 0xc4:
      case 0xc5: {  // les / lds r, m16:osz (c4 / c5 with a memory ModRM in 32-bit code; U30 for es / ds)
        if (!u.is_mem) return fault_x(L, WTFGPU_VEC_UD, 0);
        u64 off, sel;
        if (!vread(L, ea, osz, off) || !vread(L, ea + osz, 2, sel)) return X_FAULT;
        if (!load_sreg(P, L, c == 0xc4 ? WTFGPU_ES : WTFGPU_DS, (u32)sel, true)) return X_FAULT;
        setr(L, 0, u.reg, osz, off);
        return X_OK;
      }
      case 0xd6:  // salc: AL = CF ? ff : 00, flags kept
        RS(L, 0, (R(L, 0) & ~0xffull) | ((L.rflags & F_CF) ? 0xffull : 0));
        return X_OK;
      case 0xc6:  // xabort imm8: no transaction is ever active, a no-op (U48)
        return X_OK;
      case 0xc7: {  // xbegin rel32: the transaction aborts at once, EAX = 0, rip = the fallback (U48)
        if (osz == 2) return X_UNIMPL;
        const u64 target = (nrip + sext(u.imm & 0xffffffffull, 4)) & smask;
        if (!m32 && !canonical(target)) return fault_x(L, WTFGPU_VEC_GP, 0);
        RS(L, 0, 0);
        next = target;
        return X_OK;
      }
      case 0xe6: case 0xe7: case 0xee: case 0xef:  // out
        if (cpl > lane_iopl(L)) return fault_x(L, WTFGPU_VEC_GP, 0);
        return X_OK;
      case 0x8c: {  // mov r/m, Sreg
        if (r3 > 5) return fault_x(L, WTFGPU_VEC_UD, 0);
        a = r3 == WTFGPU_CS ? S.cs : r3 == WTFGPU_SS ? S.ss : F.seg[r3].selector;
        if (u.is_mem) return vwrite(L, ea, 2, a) ? X_OK : X_FAULT;
        setr(L, u.rex, u.rm, osz, a);
        return X_OK;
      }
      case 0x8e: {  // mov Sreg, r/m16
        if (r3 == WTFGPU_CS || r3 > 5) return fault_x(L, WTFGPU_VEC_UD, 0);
        if (u.is_mem) {
          if (!vread(L, ea, 2, a)) return X_FAULT;
        } else {
          a = R(L, u.rm) & 0xffff;
        }
        return load_sreg(P, L, r3, (u32)a, true) ? X_OK : X_FAULT;
      }
      case 0x9b:  // fwait (U32)
        if ((L.cr0 & 0xa) == 0xa) return fault_x(L, VEC_NM, 0);
        if (x87_pending(F)) return fault_x(L, VEC_MF, 0);
        return X_OK;
      case 0xc8: {  // enter (U29), 64-bit operand size (32-bit in 32-bit code)
        if (p66) return X_UNIMPL;
        const u64 size = u.imm & 0xffff;
        const u32 level = (u32)(u.imm >> 16) & 31;
        const u32 w = m32 ? 4 : 8;
        const u64 rsp0 = R(L, 4) & smask, rbp0 = R(L, 5) & smask;
        // written: [rsp0 - w * (level + 1), rsp0); read: [rbp0 - w * (level - 1), rbp0)
        const u32 nw = w * (level + 1);
        if (!span_w(L, (rsp0 - nw) & smask, nw)) return X_FAULT;
        u64 rsp = (rsp0 - w) & smask, rbp = rbp0;
        if (!vwrite(L, rsp, w, rbp0)) return X_FAULT;
        const u64 frame = rsp;
        if (level > 0) {
          for (u32 i = 1; i < level; i++) {
            rbp = (rbp - w) & smask;
            u64 t;
            if (!vread(L, rbp, w, t)) return X_FAULT;
            rsp = (rsp - w) & smask;
            if (!vwrite(L, rsp, w, t)) return X_FAULT;
          }
          rsp = (rsp - w) & smask;
          if (!vwrite(L, rsp, w, frame)) return X_FAULT;
        }
        RS(L, 5, frame);
        RS(L, 4, (rsp - size) & smask);
        return X_OK;
      }
      case 0xca: case 0xcb:  // far ret (U29)
        return far_pop(P, L, osz, c == 0xca ? (u.imm & 0xffff) : 0, false, m32, next);
      case 0xcf:  // iret / iretd (16- / 32-bit slots)
        return far_pop(P, L, osz, 0, true, m32, next);
      case 0xcd:  // int n (U24)
        if ((u.imm & 0xff) == 3) return X_INT3;
        return soft_int(P, L, (u32)u.imm & 0xff, true, nrip, next);
      case 0xf1:  // int1
        return soft_int(P, L, VEC_DB, false, nrip, next);
      case 0xfa: case 0xfb:  // cli / sti (U25)
        if (cpl > lane_iopl(L)) return fault_x(L, WTFGPU_VEC_GP, 0);
        if (c == 0xfa) L.rflags &= ~F_IF;
        else L.rflags |= F_IF;
        return X_OK;
      case 0xff: {  // far call / jmp m16:osz (ff /3, /5)
        if (!u.is_mem) return fault_x(L, WTFGPU_VEC_UD, 0);
        u64 off, sel;
        if (!vread(L, ea, osz, off) || !vread(L, ea + osz, 2, sel)) return X_FAULT;
        if ((sel & 0xfffc) == 0) return fault_x(L, WTFGPU_VEC_GP, 0);
        if (osz == 2) off &= 0xffff;
        if (!canonical(off)) return fault_x(L, WTFGPU_VEC_GP, 0);
        if (r3 == 3) {
          const u64 rsp = R(L, 4) & smask;
          if (!span_w(L, (rsp - 2 * osz) & smask, 2 * osz)) return X_FAULT;
          if (!vwrite(L, (rsp - osz) & smask, osz, S.cs) || !vwrite(L, (rsp - 2 * osz) & smask, osz, nrip))
            return X_FAULT;
          RS(L, 4, (rsp - 2 * osz) & smask);
        }
        set_cs(L, S, (u32)((sel & 0xfffc) | cpl));
        next = off;
        return X_OK;
      }
      default:
        if (c >= 0xd8 && c <= 0xdf) return exec_x87(P, L, u, ea);
        return X_UNIMPL;
    }
  }
  // ---- the 0f map
  switch (c) {
    case 0x00:
      if (r3 <= 1) {  // sldt / str
        if (umip && cpl) return fault_x(L, WTFGPU_VEC_GP, 0);
        a = F.seg[r3 == 0 ? WTFGPU_LDTR : WTFGPU_TR].selector;
        if (u.is_mem) return vwrite(L, ea, 2, a) ? X_OK : X_FAULT;
        setr(L, u.rex, u.rm, osz, a);
        return X_OK;
      }
      if (r3 <= 3) {  // lldt / ltr: 16-byte system descriptors of the GDT (SDM LLDT / LTR, 64-bit mode)
        if (cpl) return fault_x(L, WTFGPU_VEC_GP, 0);
        if (u.is_mem) {
          if (!vread(L, ea, 2, a)) return X_FAULT;
        } else {
          a = R(L, u.rm) & 0xffff;
        }
        const u32 sel = (u32)a & 0xffff, es = sel & 0xfffc, sr = r3 == 2 ? WTFGPU_LDTR : WTFGPU_TR;
        if (es == 0) {  // ltr: #GP(0); lldt: LDTR unusable
          if (r3 == 3) return fault_x(L, WTFGPU_VEC_GP, 0);
          F.seg[sr].selector = (u16)sel;
          F.seg[sr].present = 0;
          return X_OK;
        }
        if ((sel & 4) || (u64)(sel | 7) + 8 > F.gdtr_limit) return fault_x(L, WTFGPU_VEC_GP, es);
        const u64 da = F.gdtr_base + (sel & 0xfff8);
        if (da & 7) return X_UNIMPL;  // a misaligned GDT (U35)
        u64 d0, d1;
        if (!sup_read_q(P, L, da, d0) || !sup_read_q(P, L, da + 8, d1)) return X_FAULT;
        if (((d0 >> 40) & 0x1f) != (r3 == 2 ? 0x02u : 0x09u)) return fault_x(L, WTFGPU_VEC_GP, es);  // LDT / free TSS
        if (!((d0 >> 47) & 1)) return fault_x(L, VEC_NP, es);
        const u64 base = ((d0 >> 16) & 0xffffff) | (((d0 >> 56) & 0xff) << 24) | ((d1 & 0xffffffffull) << 32);
        if (((d1 >> 40) & 0x1f) != 0 || !canonical(base)) return fault_x(L, WTFGPU_VEC_GP, es);
        u64 lim = (d0 & 0xffff) | ((d0 >> 32) & 0xf0000);
        if ((d0 >> 55) & 1) lim = (lim << 12) | 0xfff;
        u64 nd0 = d0;
        if (r3 == 3) {  // the TSS descriptor turns busy (the last access: nothing committed before it)
          nd0 |= 2ull << 40;
          u64 ga;
          if (!sup_pa(P, L, da, 2, ga) || !sup_write_pa(P, L, ga, nd0)) return X_FAULT;
          S.tss = base;
        }
        F.seg[sr].selector = (u16)sel;
        F.seg[sr].base = base;
        F.seg[sr].limit = (u32)lim;
        F.seg[sr].attr = (u16)((nd0 >> 40) & 0xffff);
        F.seg[sr].present = 1;
        return X_OK;
      }
      if (r3 <= 5) {  // verr / verw
        if (u.is_mem) {
          if (!vread(L, ea, 2, a)) return X_FAULT;
        } else {
          a = R(L, u.rm) & 0xffff;
        }
        u64 dsc = 0;
        const int rc = gdt_desc(P, L, (u32)a, dsc);
        if (rc < 0) return X_FAULT;
        bool ok = false;
        if (rc == 0) {
          const u32 type = (u32)(dsc >> 40) & 0xf, s = (u32)(dsc >> 44) & 1, dpl = (u32)(dsc >> 45) & 3;
          const u32 rpl = (u32)a & 3, code = (type >> 3) & 1, conforming = code && ((type >> 2) & 1);
          const bool priv = conforming || (dpl >= cpl && dpl >= rpl);
          if (s && priv) ok = r3 == 4 ? (!code || (type & 2)) : (!code && (type & 2));
        }
        L.rflags = (L.rflags & ~F_ZF) | (ok ? F_ZF : 0);
        return X_OK;
      }
      return fault_x(L, WTFGPU_VEC_UD, 0);
    case 0x01:
      if (u.is_mem) {
        if (r3 <= 1) {  // sgdt / sidt
          if (umip && cpl) return fault_x(L, WTFGPU_VEC_GP, 0);
          const u64 lim = r3 == 0 ? F.gdtr_limit : S.idtr_limit;
          const u64 base = r3 == 0 ? F.gdtr_base : F.idtr_base;
          if (!span_w(L, ea, 10)) return X_FAULT;
          if (!vwrite(L, ea, 2, lim & 0xffff) || !vwrite(L, ea + 2, 8, base)) return X_FAULT;
          return X_OK;
        }
        if (r3 <= 3) {  // lgdt / lidt
          if (cpl) return fault_x(L, WTFGPU_VEC_GP, 0);
          u64 lim, base;
          if (!vread(L, ea, 2, lim) || !vread(L, ea + 2, 8, base)) return X_FAULT;
          if (!canonical(base)) return fault_x(L, WTFGPU_VEC_GP, 0);
          if (r3 == 2) {
            F.gdtr_base = base;
            F.gdtr_limit = (u32)lim;
          } else {
            F.idtr_base = base;
            F.idtr_limit = (u32)lim;
            S.idtr = base;
            S.idtr_limit = (u32)lim;
          }
          return X_OK;
        }
        if (r3 == 4) {  // smsw m16
          if (umip && cpl) return fault_x(L, WTFGPU_VEC_GP, 0);
          return vwrite(L, ea, 2, L.cr0 & 0xffff) ? X_OK : X_FAULT;
        }
        if (r3 == 6) {  // lmsw m16
          if (cpl) return fault_x(L, WTFGPU_VEC_GP, 0);
          if (!vread(L, ea, 2, a)) return X_FAULT;
        } else if (r3 == 7) {  // invlpg
          if (cpl) return fault_x(L, WTFGPU_VEC_GP, 0);
          L.flush = 1;
          return X_OK;
        } else {
          return fault_x(L, WTFGPU_VEC_UD, 0);
        }
      } else {
        const u32 modrm = 0xc0 | (r3 << 3) | (u.rm & 7);
        if (r3 == 4) {  // smsw r
          if (umip && cpl) return fault_x(L, WTFGPU_VEC_GP, 0);
          setr(L, u.rex, u.rm, osz, osz == 2 ? (L.cr0 & 0xffff) : (L.cr0 & 0xffffffffull));
          return X_OK;
        }
        if (modrm == 0xd0 || modrm == 0xd1) {  // xgetbv / xsetbv (U27)
          if (!((S.cr4 >> 18) & 1)) return fault_x(L, WTFGPU_VEC_UD, 0);
          if ((u32)R(L, 1) != 0) return fault_x(L, WTFGPU_VEC_GP, 0);
          if (modrm == 0xd0) {
            RS(L, 0, F.xcr0 & 0xffffffffull);
            RS(L, 2, F.xcr0 >> 32);
            return X_OK;
          }
          const u64 v = (R(L, 0) & 0xffffffffull) | (R(L, 2) << 32);
          // (bits 7:5, the AVX-512 state, all or none and only with 2:1 = 11)
          if (cpl || (v & ~XS_SUPPORTED) || !(v & 1) || ((v & 4) && !(v & 2)) || (((v >> 3) & 1) != ((v >> 4) & 1)) ||
              ((v & 0xe0) && ((v & 0xe0) != 0xe0 || (v & 6) != 6)))
            return fault_x(L, WTFGPU_VEC_GP, 0);
          F.xcr0 = v;
          L.simd = simd_bits(L.cr0, S.cr4, v);
          return X_OK;
        }
        if (modrm == 0xd5) return fault_x(L, WTFGPU_VEC_GP, 0);  // xend outside a transaction (U48)
        if (modrm == 0xd6) {                                     // xtest: never in a transaction
          L.rflags = (L.rflags & ~F_STATUS) | F_ZF;
          return X_OK;
        }
        if (r3 != 6) return fault_x(L, WTFGPU_VEC_UD, 0);
        if (cpl) return fault_x(L, WTFGPU_VEC_GP, 0);  // lmsw r
        a = R(L, u.rm) & 0xffff;
      }
      // lmsw: PE (set only), MP, EM, TS
      L.cr0 = S.cr0 = (L.cr0 & ~0xeull) | (a & 0xf) | (L.cr0 & 1);
      L.simd = simd_bits(L.cr0, S.cr4, F.xcr0);
      return X_OK;
    case 0x02:
    case 0x03: {  // lar / lsl
      if (u.is_mem) {
        if (!vread(L, ea, 2, a)) return X_FAULT;
      } else {
        a = R(L, u.rm) & 0xffff;
      }
      u64 dsc = 0;
      const int rc = gdt_desc(P, L, (u32)a, dsc);
      if (rc < 0) return X_FAULT;
      bool ok = false;
      if (rc == 0) {
        const u32 type = (u32)(dsc >> 40) & 0xf, s = (u32)(dsc >> 44) & 1, dpl = (u32)(dsc >> 45) & 3;
        const u32 rpl = (u32)a & 3, conforming = s && (type & 0xc) == 0xc;
        const bool sys_ok = !s && (type == 2 || type == 9 || type == 0xb || (c == 0x02 && type == 0xc));
        ok = (s || sys_ok) && (conforming || (dpl >= cpl && dpl >= rpl));
      }
      if (ok) {
        u64 v;
        if (c == 0x02) {
          v = (dsc >> 32) & 0x00f0ff00ull;
        } else {
          v = (dsc & 0xffff) | ((dsc >> 32) & 0xf0000);
          if ((dsc >> 55) & 1) v = (v << 12) | 0xfff;
        }
        setr(L, u.rex, u.reg, osz, v & szmask(osz));
      }
      L.rflags = (L.rflags & ~F_ZF) | (ok ? F_ZF : 0);
      return X_OK;
    }
    case 0x06:  // clts
      if (cpl) return fault_x(L, WTFGPU_VEC_GP, 0);
      L.cr0 = S.cr0 = L.cr0 & ~8ull;
      L.simd = simd_bits(L.cr0, S.cr4, F.xcr0);
      return X_OK;
    case 0x08:
    case 0x09:  // invd / wbinvd
      return cpl ? fault_x(L, WTFGPU_VEC_GP, 0) : X_OK;
    case 0x21:
    case 0x23: {  // mov r64, drN / mov drN, r64: reads 0, writes dropped (U35)
      const u32 n = u.reg & 15;
      if (n > 7 || ((n == 4 || n == 5) && ((S.cr4 >> 3) & 1))) return fault_x(L, WTFGPU_VEC_UD, 0);
      if (cpl) return fault_x(L, WTFGPU_VEC_GP, 0);
      if (c == 0x21) RS(L, u.rm, 0);
      return X_OK;
    }
    case 0x33:  // rdpmc
      if ((cpl && !((S.cr4 >> 8) & 1)) || (u32)R(L, 1) > 3) return fault_x(L, WTFGPU_VEC_GP, 0);
      RS(L, 0, 0);
      RS(L, 2, 0);
      return X_OK;
    case 0x34:  // sysenter
      if ((F.sysenter_cs & 0xfffc) == 0) return fault_x(L, WTFGPU_VEC_GP, 0);
      L.rflags &= ~(0x20000ull | 0x200ull | 0x10000ull);
      set_cs(L, S, (u32)(F.sysenter_cs & 0xfffc));
      S.ss = (u16)((F.sysenter_cs & 0xfffc) + 8);
      if (cpl != 0) L.flush = 1;
      L.cpl = S.cpl = 0;
      RS(L, 4, F.sysenter_esp);
      next = F.sysenter_eip;
      return X_OK;
    case 0x35:  // sysexit (64-bit form)
      if (!rexw) return X_UNIMPL;
      if ((F.sysenter_cs & 0xfffc) == 0 || cpl) return fault_x(L, WTFGPU_VEC_GP, 0);
      if (!canonical(R(L, 2)) || !canonical(R(L, 1))) return fault_x(L, WTFGPU_VEC_GP, 0);
      set_cs(L, S, (u32)(((F.sysenter_cs + 32) & 0xfffc) | 3));
      S.ss = (u16)(((F.sysenter_cs + 40) & 0xfffc) | 3);
      L.flush = 1;
      L.cpl = S.cpl = 3;
      RS(L, 4, R(L, 1));
      next = R(L, 2);
      return X_OK;
    case 0xa0:
    case 0xa8: {  // push fs / gs
      const u32 sz = u.bsz;  // the stack slot
      if (!vwrite(L, ((R(L, 4) & smask) - sz) & smask, sz, F.seg[c == 0xa0 ? WTFGPU_FS : WTFGPU_GS].selector))
        return X_FAULT;
      RS(L, 4, ((R(L, 4) & smask) - sz) & smask);
      return X_OK;
    }
    case 0xa1:
    case 0xa9: {  // pop fs / gs
      const u32 sz = u.bsz;  // the stack slot
      if (!vread(L, R(L, 4) & smask, sz, a)) return X_FAULT;
      if (!load_sreg(P, L, c == 0xa1 ? WTFGPU_FS : WTFGPU_GS, (u32)a & 0xffff, true)) return X_FAULT;
      RS(L, 4, ((R(L, 4) & smask) + sz) & smask);
      return X_OK;
    }
    case 0xa2: {  // cpuid (U27)
      u32 r[4];
      cpuid_leaf(S.cr4, F.xcr0, (u32)R(L, 0), (u32)R(L, 1), r);
      RS(L, 0, r[0]);
      RS(L, 3, r[1]);
      RS(L, 1, r[2]);
      RS(L, 2, r[3]);
      return X_OK;
    }
    case 0xb2:
    case 0xb4:
    case 0xb5: {  // lss / lfs / lgs m16:osz
      if (!u.is_mem) return fault_x(L, WTFGPU_VEC_UD, 0);
      u64 off, sel;
      if (!vread(L, ea, osz, off) || !vread(L, ea + osz, 2, sel)) return X_FAULT;
      const u32 sr = c == 0xb2 ? WTFGPU_SS : c == 0xb4 ? WTFGPU_FS : WTFGPU_GS;
      if (!load_sreg(P, L, sr, (u32)sel, true)) return X_FAULT;
      setr(L, u.rex, u.reg, osz, off);
      return X_OK;
    }
    case 0xae:  // group 15 beyond ldmxcsr / stmxcsr / the fences
      if (u.is_mem) {
        if (u.rep) return fault_x(L, WTFGPU_VEC_UD, 0);
        if (p66 && r3 != 6 && r3 != 7) return fault_x(L, WTFGPU_VEC_UD, 0);
        if (!p66) {
          if (r3 == 0 || r3 == 1) return fxsave_op(P, L, r3 == 1, ea);
          if (r3 == 4) return xsave_op(P, L, XS_SAVE, ea);
          if (r3 == 5) return xsave_op(P, L, XS_RSTOR, ea);
          if (r3 == 6) return xsave_op(P, L, XS_SAVEOPT, ea);
          if (r3 != 7) return fault_x(L, WTFGPU_VEC_UD, 0);
        }
        // clflush / clflushopt / clwb: a read translation, no bytes
        if (!xlate(L, ea, ACC_R)) return X_FAULT;
        return X_OK;
      }
      if (u.rep == 0xf3 && !p66 && r3 <= 3) {  // rd / wr fs / gs base
        if (!((S.cr4 >> 16) & 1)) return fault_x(L, WTFGPU_VEC_UD, 0);
        const u32 sz = rexw ? 8 : 4;
        u64 *bp = (r3 & 1) ? P.gs_base : P.fs_base;
        if (r3 <= 1) {
          setr(L, u.rex, u.rm, sz, bp[L.lane]);
        } else {
          a = R(L, u.rm) & szmask(sz);
          if (!canonical(a)) return fault_x(L, WTFGPU_VEC_GP, 0);
          bp[L.lane] = a;
        }
        return X_OK;
      }
      return fault_x(L, WTFGPU_VEC_UD, 0);
    case 0xc7:
      if (u.is_mem && r3 == 1 && !u.rep && !p66) {  // cmpxchg8b / cmpxchg16b (U28)
        u64 v0, v1 = 0;
        if (rexw) {
          if (ea & 15) return fault_x(L, WTFGPU_VEC_GP, 0);
          if (!vread(L, ea, 8, v0, ACC_W) || !vread(L, ea + 8, 8, v1, ACC_W)) return X_FAULT;
          const bool eq = v0 == R(L, 0) && v1 == R(L, 2);
          if (!vwrite(L, ea, 8, eq ? R(L, 3) : v0) || !vwrite(L, ea + 8, 8, eq ? R(L, 1) : v1)) return X_FAULT;
          if (!eq) {
            RS(L, 0, v0);
            RS(L, 2, v1);
          }
          L.rflags = (L.rflags & ~F_ZF) | (eq ? F_ZF : 0);
        } else {
          if (!vread(L, ea, 8, v0, ACC_W)) return X_FAULT;
          const u64 cur = (R(L, 0) & 0xffffffffull) | (R(L, 2) << 32);
          const bool eq = v0 == cur;
          if (!vwrite(L, ea, 8, eq ? ((R(L, 3) & 0xffffffffull) | (R(L, 1) << 32)) : v0)) return X_FAULT;
          if (!eq) {
            RS(L, 0, v0 & 0xffffffffull);
            RS(L, 2, v0 >> 32);
          }
          L.rflags = (L.rflags & ~F_ZF) | (eq ? F_ZF : 0);
        }
        return X_OK;
      }
      if (u.is_mem && !u.rep && !p66 && (r3 == 3 || r3 == 4 || r3 == 5))
        return xsave_op(P, L, r3 == 3 ? XS_RSTORS : r3 == 4 ? XS_SAVEC : XS_SAVES, ea);
      return fault_x(L, WTFGPU_VEC_UD, 0);
    default:
      return fault_x(L, WTFGPU_VEC_UD, 0);
  }
}

}  // namespace wtfgpu_dev
