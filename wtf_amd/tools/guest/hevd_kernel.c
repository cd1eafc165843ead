/* hevd kernel guest — the ring-0 half of the synthetic HEVD snapshot.
 *
 * No HEVD snapshot (a Windows kernel + HackSysExtremeVulnerableDriver memory
 * dump) can be fetched offline. This is a freestanding
 * look-alike of what the reference's fuzzer_hevd module drives
 * (src/wtf/fuzzer_hevd.cc): a user-mode DeviceIoControl call reaches the
 * kernel through SYSCALL, the system-call entry switches to the kernel stack
 * (SWAPGS + per-processor block), and an IOCTL dispatcher runs handlers
 * modelled on HEVD's classic bug classes:
 *   0x222003 stack buffer overflow (no cookie: the return address is overrun)
 *   0x222007 stack buffer overflow with a /GS cookie -> KeBugCheck2(0xF7)
 *   0x22200B arbitrary write (write-what-where from user pointers)
 *   0x22200F pool overflow -> pool header check on free -> KeBugCheck2(0x19)
 *   0x222013 null pointer dereference (callback through a NULL object)
 *   0x222017 integer overflow of a size check -> GS-protected copy
 *   0x22201B type confusion (calls a function pointer taken from user data)
 *   0x22201F wait on an object -> nt!SwapContext (context switch)
 * Every handler logs through nt!DbgPrintEx, and the pool cookie comes from
 * nt!ExGenRandom, whose `rdrand rdx` sits at +0xe0 like the Windows build the
 * module checks (fuzzer_hevd.cc:96-101), mixed with the time-stamp counter.
 * As in HEVD, the handlers touch user memory inside __try / __except: a page
 * fault on a user address there is dispatched to the handler (the trap
 * returns through IRETQ into the guarded function's except path with
 * STATUS_ACCESS_VIOLATION); a fault on a kernel address bugchecks.
 *
 * Compiled with gcc (-mabi=ms: Win64 argument registers) into a flat image at
 * KERNEL_BASE, mapped supervisor-only by wtf_amd/tools/hevd.py.
 *
 * Built with -DHEVD_IO (the "hevd_io" workload, wtf_amd/tools/hevd.py), the
 * request takes the path Windows gives a METHOD_NEITHER DeviceIoControl
 * instead of a direct call: a trap frame in KiSystemCall64, the handle
 * resolved through the process handle table to a referenced file object
 * (ObReferenceObjectByHandle), an IRP from a lookaside list with one stack
 * location per device of the stack (IoAllocateIrp), the thread's IRP list,
 * IofCallDriver through a filter device (which copies its stack location
 * down and sets a completion routine) to HEVD's IrpDeviceIoCtlHandler via the
 * driver object's MajorFunction table, and IofCompleteRequest (completion
 * routines bottom-up, the I/O status block copied to the caller, the event
 * signalled, the IRP back on its list, the file object dereferenced). The
 * driver also answers four benign requests HEVD-style drivers carry (a CRC
 * over the input, a record parser, a bounded copy, a command list over a
 * kernel table), the common traffic of the variant's seed corpus.
 */
#include "sse_rt.h"
typedef unsigned long long u64;
typedef unsigned int u32;
typedef unsigned short u16;
typedef unsigned char u8;

#define STATUS_SUCCESS 0u
#define STATUS_INVALID_DEVICE_REQUEST 0xC0000010u
#define STATUS_UNSUCCESSFUL 0xC0000001u

/* ---- freestanding helpers (gcc may emit calls to these) */
__attribute__((used)) void *memcpy(void *d, const void *s, u64 n) {
  sse_copy(d, s, n);
  return d;
}
__attribute__((used)) void *memset(void *d, int c, u64 n) {
  sse_fill(d, c, n);
  return d;
}

/* ---- nt exports the module breakpoints (bodies are never reached) */
__attribute__((noipa, used)) u32 DbgPrintEx(u32 ComponentId, u32 Level, const char *Format, ...) {
  (void)ComponentId, (void)Level, (void)Format;
  return 0;
}
__attribute__((noipa, used, naked)) void KeBugCheck2(u64 Code, u64 P1, u64 P2, u64 P3, u64 P4, u64 P5) {
  __asm__ volatile("hlt");
}
__attribute__((noipa, used, naked)) void SwapContext(void) { __asm__ volatile("hlt"); }

/* ExGenRandom: `rdrand rdx` at +0xe0 (48 0f c7 f2); the module's breakpoint
 * right after it replaces rdx with Backend_t::Rdrand(). */
__asm__(".globl ExGenRandom\n"
        ".p2align 4\n"
        "ExGenRandom:\n"
        "  jmp 1f\n"            /* e9 rel32 */
        "  .fill 0xdb, 1, 0xcc\n"
        "1: rdrand %rdx\n"
        "  mov %rdx, %rax\n"
        "  ret\n");
u64 ExGenRandom(void);

/* KeBugCheckEx -> KeBugCheck2 with the Win64 argument shape the module reads
 * (GetArg(0..5): rcx, rdx, r8, r9, [rsp+0x28], [rsp+0x30]). */
__attribute__((noipa, noreturn)) void KeBugCheckEx(u64 Code, u64 P1, u64 P2, u64 P3, u64 P4) {
  KeBugCheck2(Code, P1, P2, P3, P4, 0);
  for (;;) __asm__ volatile("hlt");
}

/* ---- __try / __except: a guarded region registers its resume context; the
 * page-fault path (KiTrapHandler) sends a user-address fault inside it to
 * KiTryResume through IRETQ, which unwinds to the region's except path. */
#define STATUS_ACCESS_VIOLATION 0xC0000005u
typedef struct {
  void *Jmp[5];
} KTRY;
static KTRY *volatile CurrentTry;
__attribute__((noipa, used)) void KiTryResume(void) { __builtin_longjmp(CurrentTry->Jmp, 1); }
/* the barriers keep the guarded accesses between the two stores */
static inline __attribute__((always_inline)) int TryEnter(KTRY *T) {
  CurrentTry = T;
  __asm__ volatile("" ::: "memory");
  return 1;
}
static inline __attribute__((always_inline)) void TryLeave(void) {
  __asm__ volatile("" ::: "memory");
  CurrentTry = 0;
}
#define TRY(T) if (__builtin_setjmp((T).Jmp) == 0 && TryEnter(&(T)))
#define EXCEPT else
#define END_TRY() TryLeave()

/* ---- /GS cookie */
u64 __security_cookie = 0x00002B992DDFA232ull;
__attribute__((noipa)) static void CheckCookie(u64 Saved, u64 Frame) {
  if ((Saved ^ Frame) != __security_cookie) KeBugCheckEx(0xF7, Saved ^ Frame, __security_cookie, ~__security_cookie, 0);
}

/* ---- a small nonpaged pool: chunks with a 16-byte header */
struct PoolHeader {
  u32 Size;
  u32 Tag;
  u64 Cookie;
};
#define POOL_SIZE 0x3000
struct {
  u64 Cursor;
  u64 Cookie;
  u8 Arena[POOL_SIZE];
} Pool;

static u64 PoolCookie(void) {
  if (!Pool.Cookie) {
    u32 lo, hi;
    __asm__ volatile("rdtsc" : "=a"(lo), "=d"(hi));
    Pool.Cookie = (ExGenRandom() ^ ((u64)hi << 32 | lo)) | 1;
  }
  return Pool.Cookie;
}
__attribute__((noipa)) void *ExAllocatePoolWithTag(u32 Type, u64 Size, u32 Tag) {
  (void)Type;
  Size = (Size + 15) & ~15ull;
  if (Pool.Cursor + sizeof(struct PoolHeader) + Size > POOL_SIZE) return 0;
  struct PoolHeader *H = (struct PoolHeader *)(Pool.Arena + Pool.Cursor);
  H->Size = (u32)Size;
  H->Tag = Tag;
  H->Cookie = PoolCookie() ^ (u64)H;
  Pool.Cursor += sizeof(struct PoolHeader) + Size;
  /* the next chunk header is written now so an overflow lands on it */
  struct PoolHeader *N = (struct PoolHeader *)(Pool.Arena + Pool.Cursor);
  if (Pool.Cursor + sizeof(struct PoolHeader) <= POOL_SIZE) {
    N->Size = 0;
    N->Tag = 0x65657246; /* 'Free' */
    N->Cookie = PoolCookie() ^ (u64)N;
  }
  return H + 1;
}
__attribute__((noipa)) void ExFreePoolWithTag(void *P, u32 Tag) {
  struct PoolHeader *H = (struct PoolHeader *)P - 1;
  struct PoolHeader *N = (struct PoolHeader *)((u8 *)P + H->Size);
  if (H->Tag != Tag || (H->Cookie ^ (u64)H) != PoolCookie()) KeBugCheckEx(0x19, 0x20, (u64)H, (u64)N, H->Cookie);
  if ((u8 *)N + sizeof(*N) <= Pool.Arena + POOL_SIZE && (N->Cookie ^ (u64)N) != PoolCookie())
    KeBugCheckEx(0x19, 0x21, (u64)H, (u64)N, N->Cookie); /* BAD_POOL_HEADER: next chunk overrun */
}

/* ---- the IOCTL handlers */
#define TAG 0x6B636148 /* 'Hack' */

struct GsFrame {
  u8 Kernel[512];
  u64 Cookie;
};
#ifdef HEVD_IO
/* (HEVD_IO: built with /GS like the rest of the driver, so an overrun is
 * caught by the cookie check before the return address is used: a bugcheck
 * instead of a return into arbitrary kernel code) */
__attribute__((noipa)) static u32 TriggerBufferOverflowStack(const u8 *User, u64 Size) {
  struct GsFrame F;
  KTRY T;
  F.Cookie = __security_cookie ^ (u64)&F;
  memset(F.Kernel, 0, sizeof(F.Kernel));
  DbgPrintEx(77, 3, "[+] UserBuffer: 0x%p Size: 0x%zX\n", User, Size);
  u32 Status = F.Kernel[0] == 0x41 ? STATUS_SUCCESS : STATUS_UNSUCCESSFUL;
  TRY(T) {
    memcpy(F.Kernel, User, Size); /* the bug: Size is the user's, not sizeof(Kernel) */
    END_TRY();
    Status = F.Kernel[0] == 0x41 ? STATUS_SUCCESS : STATUS_UNSUCCESSFUL;
  }
  EXCEPT {
    END_TRY();
    Status = STATUS_ACCESS_VIOLATION;
  }
  CheckCookie(F.Cookie, (u64)&F);
  return Status;
}
#else
__attribute__((noipa)) static u32 TriggerBufferOverflowStack(const u8 *User, u64 Size) {
  u8 Kernel[512];
  KTRY T;
  memset(Kernel, 0, sizeof(Kernel));
  DbgPrintEx(77, 3, "[+] UserBuffer: 0x%p Size: 0x%zX\n", User, Size);
  TRY(T) {
    memcpy(Kernel, User, Size); /* the bug: Size is the user's, not sizeof(Kernel) */
    END_TRY();
  }
  EXCEPT {
    END_TRY();
    return STATUS_ACCESS_VIOLATION;
  }
  return Kernel[0] == 0x41 ? STATUS_SUCCESS : STATUS_UNSUCCESSFUL;
}
#endif

__attribute__((noipa)) static u32 TriggerBufferOverflowStackGS(const u8 *User, u64 Size) {
  struct GsFrame F;
  F.Cookie = __security_cookie ^ (u64)&F;
  memset(F.Kernel, 0, sizeof(F.Kernel));
  DbgPrintEx(77, 3, "[+] GS UserBuffer: 0x%p Size: 0x%zX\n", User, Size);
  memcpy(F.Kernel, User, Size);
  CheckCookie(F.Cookie, (u64)&F);
  return STATUS_SUCCESS;
}

struct WhatWhere {
  u64 *What;
  u64 *Where;
};
__attribute__((noipa)) static u32 TriggerArbitraryWrite(const u8 *User, u64 Size) {
  if (Size < sizeof(struct WhatWhere)) return STATUS_UNSUCCESSFUL;
  const struct WhatWhere *W = (const struct WhatWhere *)User;
  KTRY T;
  DbgPrintEx(77, 3, "[+] What: 0x%p Where: 0x%p\n", W->What, W->Where);
  TRY(T) {
    *(W->Where) = *(W->What);
    END_TRY();
  }
  EXCEPT {
    END_TRY();
    return STATUS_ACCESS_VIOLATION;
  }
  return STATUS_SUCCESS;
}

__attribute__((noipa)) static u32 TriggerPoolOverflow(const u8 *User, u64 Size) {
  u8 *Chunk = ExAllocatePoolWithTag(0, 0x1f8, TAG);
  if (!Chunk) return STATUS_UNSUCCESSFUL;
  KTRY T;
  DbgPrintEx(77, 3, "[+] Pool chunk: 0x%p Size: 0x%zX\n", Chunk, Size);
  TRY(T) {
    memcpy(Chunk, User, Size);
    END_TRY();
  }
  EXCEPT {
    END_TRY();
    return STATUS_ACCESS_VIOLATION;
  }
  ExFreePoolWithTag(Chunk, TAG);
  return STATUS_SUCCESS;
}

struct NullObject {
  u64 Value;
  void (*Callback)(void);
};
static void NullCallback(void) { DbgPrintEx(77, 3, "[+] Callback\n"); }
__attribute__((noipa)) static u32 TriggerNullPointerDereference(const u8 *User, u64 Size) {
  if (Size < 4) return STATUS_UNSUCCESSFUL;
  struct NullObject *volatile Obj = ExAllocatePoolWithTag(0, sizeof(struct NullObject), TAG);
  if (!Obj) return STATUS_UNSUCCESSFUL;
  Obj->Value = 0xBAD0B0B0;
  Obj->Callback = NullCallback;
  if (*(const u32 *)User == 0xBAD0B0B0) {
    DbgPrintEx(77, 3, "[+] Freeing the object\n");
    ExFreePoolWithTag(Obj, TAG);
    Obj = 0; /* the bug: the object is used after this */
  }
  Obj->Callback();
  return STATUS_SUCCESS;
}

__attribute__((noipa)) static u32 TriggerIntegerOverflow(const u8 *User, u64 Size) {
  struct GsFrame F;
  F.Cookie = __security_cookie ^ (u64)&F;
  const u32 Terminator = 0xBAD0B0B0;
  if (Size < 4) return STATUS_UNSUCCESSFUL;
  const u32 Declared = *(const u32 *)User; /* the request's own length field */
  DbgPrintEx(77, 3, "[+] Integer overflow Declared: 0x%X\n", Declared);
  if ((u32)(Declared + 4) > sizeof(F.Kernel)) return STATUS_UNSUCCESSFUL; /* the bug: 32-bit wrap */
  const u32 *Words = (const u32 *)(User + 4);
  for (u64 i = 0; i < Declared / 4; i++) {
    if (Words[i] == Terminator) break;
    ((u32 *)F.Kernel)[i] = Words[i];
  }
  CheckCookie(F.Cookie, (u64)&F);
  return STATUS_SUCCESS;
}

struct TypeConfusionObject {
  u64 ObjectId;
  union {
    u64 ObjectType;
    void (*Callback)(void);
  };
};
__attribute__((noipa)) static u32 TriggerTypeConfusion(const u8 *User, u64 Size) {
  if (Size < sizeof(struct TypeConfusionObject)) return STATUS_UNSUCCESSFUL;
  struct TypeConfusionObject *K = ExAllocatePoolWithTag(0, sizeof(*K), TAG);
  if (!K) return STATUS_UNSUCCESSFUL;
  memcpy(K, User, sizeof(*K));
  DbgPrintEx(77, 3, "[+] ObjectId: 0x%p ObjectType: 0x%p\n", K->ObjectId, K->ObjectType);
  if (K->ObjectId == 0x4242424242424242ull) K->Callback(); /* the bug: the type field is called */
  ExFreePoolWithTag(K, TAG);
  return STATUS_SUCCESS;
}

__attribute__((noipa)) static u32 TriggerWait(const u8 *User, u64 Size) {
  if (Size >= 8 && *(const u64 *)User == 0x5741495457414954ull) { /* "TIAWTIAW" */
    DbgPrintEx(77, 3, "[+] Waiting\n");
    ((void (*)(void))SwapContext)(); /* KeWaitForSingleObject -> context switch */
  }
  return STATUS_SUCCESS;
}

#ifdef HEVD_IO
/* ---- benign requests (HEVD_IO): the variant's common traffic */
#define STATUS_INVALID_PARAMETER 0xC000000Du
static const u32 Crc32Nibble[16] = {0x00000000u, 0x1DB71064u, 0x3B6E20C8u, 0x26D930ACu, 0x76DC4190u, 0x6B6B51F4u,
                                    0x4DB26158u, 0x5005713Cu, 0xEDB88320u, 0xF00F9344u, 0xD6D6A3E8u, 0xCB61B38Cu,
                                    0x9B64C2B0u, 0x86D3D2D4u, 0xA00AE278u, 0xBDBDF21Cu};
/* ProbeForRead: range inside user space, then one read per page */
#define MM_USER_PROBE_ADDRESS 0x7FFFFFFF0000ull
static void ExRaiseAccessViolation(void) { *(volatile u8 *)0x7FFFFFFF0000ull; }
__attribute__((noipa)) static void ProbeForRead(const u8 *P, u64 Size, u32 Align) {
  if (!Size) return;
  if (((u64)P & (Align - 1)) || (u64)P + Size < (u64)P || (u64)P + Size > MM_USER_PROBE_ADDRESS)
    ExRaiseAccessViolation();
  for (u64 Page = (u64)P & ~0xFFFull; Page < (u64)P + Size; Page += 0x1000) (void)*(volatile const u8 *)Page;
}
static u64 LastInformation;
__attribute__((noipa)) static u32 TriggerChecksum(const u8 *User, u64 Size) {
  KTRY T;
  u32 Crc = 0xFFFFFFFFu;
  TRY(T) {
    ProbeForRead(User, Size, 1);
    for (u64 i = 0; i < Size; i++) {
      Crc ^= User[i];
      Crc = (Crc >> 4) ^ Crc32Nibble[Crc & 15];
      Crc = (Crc >> 4) ^ Crc32Nibble[Crc & 15];
    }
    END_TRY();
  }
  EXCEPT {
    END_TRY();
    return STATUS_ACCESS_VIOLATION;
  }
  LastInformation = ~Crc;
  DbgPrintEx(77, 3, "[+] Checksum: 0x%X\n", ~Crc);
  return STATUS_SUCCESS;
}
/* records: [u16 length][u8 type][payload], each folded into a kernel table */
static struct {
  u32 Count[16];
  u64 Sum[16];
} RecordStats;
__attribute__((noipa)) static u32 TriggerParseRecords(const u8 *User, u64 Size) {
  u8 Kernel[1024];
  if (Size > sizeof(Kernel)) return STATUS_INVALID_PARAMETER;
  KTRY T;
  TRY(T) {
    ProbeForRead(User, Size, 1);
    memcpy(Kernel, User, Size);
    END_TRY();
  }
  EXCEPT {
    END_TRY();
    return STATUS_ACCESS_VIOLATION;
  }
  u64 At = 0, N = 0;
  while (At + 3 <= Size) {
    const u32 Len = Kernel[At] | (u32)Kernel[At + 1] << 8, Type = Kernel[At + 2] & 15;
    if (Len < 3 || At + Len > Size) return STATUS_INVALID_PARAMETER;
    /* each record type has its own fold (a parser's per-type handlers) */
    const u8 *Pl = Kernel + At + 3;
    const u32 Pn = Len - 3;
    u64 Sum = 0;
    switch (Type) {
      case 0: for (u32 i = 0; i < Pn; i++) Sum += Pl[i]; break;
      case 1: for (u32 i = 0; i < Pn; i++) Sum ^= (u64)Pl[i] << (8 * (i & 7)); break;
      case 2: for (u32 i = 0; i < Pn; i++) Sum = Pl[i] > Sum ? Pl[i] : Sum; break;
      case 3: for (u32 i = 0; i < Pn; i++) Sum += Pl[i] != 0; break;
      case 4: for (u32 i = 0; i < Pn; i++) Sum = (Sum << 5 | Sum >> 59) ^ Pl[i]; break;
      case 5: for (u32 i = 0; i + 1 < Pn; i += 2) Sum += (u32)(Pl[i] | Pl[i + 1] << 8); break;
      case 6: for (u32 i = 0; i < Pn; i++) for (u32 b = Pl[i]; b; b &= b - 1) Sum++; break;
      case 7: for (u32 i = 0; i < Pn; i++) Sum = Sum * 131 + (Pl[i] | 0x20); break;
      case 8: for (u32 i = 0; i < Pn; i++) if (Pl[i] >= '0' && Pl[i] <= '9') Sum = Sum * 10 + (Pl[i] - '0'); break;
      case 9: for (u32 i = 0; i < Pn; i++) Sum += (Pl[i] & 0x80) ? 1 : 0; break;
      case 10: for (u32 i = 0; i + 3 < Pn; i += 4) Sum ^= *(const u32 *)(Pl + i); break;
      case 11: for (u32 i = 0; i < Pn; i++) Sum = (Sum + Pl[i]) % 65521; break;
      case 12: for (u32 i = Pn; i > 0; i--) Sum = Sum * 7 + Pl[i - 1]; break;
      case 13: for (u32 i = 0; i < Pn; i++) Sum |= 1ull << (Pl[i] & 63); break;
      case 14: for (u32 i = 0; i < Pn; i++) Sum += (u64)Pl[i] * (i + 1); break;
      default: for (u32 i = 0; i < Pn; i++) Sum = Sum * 31 + Pl[i]; break;
    }
    RecordStats.Count[Type]++;
    RecordStats.Sum[Type] += Sum;
    At += Len;
    N++;
  }
  LastInformation = N;
  return At == Size ? STATUS_SUCCESS : STATUS_INVALID_PARAMETER;
}
/* a command list over a small kernel table: [u8 op][u8 a][u8 b][u8 c] per
 * command, each op its own routine with its own argument checks (a driver's
 * control interface) */
static u64 CmdTable[64];
typedef u32 (*CmdFn)(u32 A, u32 B, u32 C);
#define CMD(n, ...) static u32 Cmd##n(u32 A, u32 B, u32 C) { (void)A, (void)B, (void)C; __VA_ARGS__ }
CMD(0, { CmdTable[A & 63] = B | C << 8; return 0; })
CMD(1, { return (u32)CmdTable[A & 63]; })
CMD(2, { CmdTable[A & 63] += CmdTable[B & 63]; return 0; })
CMD(3, { CmdTable[A & 63] ^= (u64)B << (C & 56); return 0; })
CMD(4, { if (A >= 64 || B >= 64 || A > B) return 1; u64 S = 0; for (u32 i = A; i <= B; i++) S += CmdTable[i]; CmdTable[C & 63] = S; return 0; })
CMD(5, { if (A >= 64) return 1; CmdTable[A] = CmdTable[A] << (B & 63) | CmdTable[A] >> (64 - (B & 63) & 63); return 0; })
CMD(6, { if (A >= 64 || B >= 64) return 1; u64 T = CmdTable[A]; CmdTable[A] = CmdTable[B]; CmdTable[B] = T; return 0; })
CMD(7, { if (A >= 64 || B >= 64 || A > B) return 1; for (u32 i = A; i < B; i++) for (u32 j = i + 1; j <= B; j++) if (CmdTable[j] < CmdTable[i]) { u64 T = CmdTable[i]; CmdTable[i] = CmdTable[j]; CmdTable[j] = T; } return 0; })
CMD(8, { if (!B) return 1; CmdTable[A & 63] /= B; return 0; })
CMD(9, { if (!B) return 1; CmdTable[A & 63] %= B; return 0; })
CMD(10, { CmdTable[A & 63] = CmdTable[A & 63] * (B | 1) + C; return 0; })
CMD(11, { return CmdTable[A & 63] > CmdTable[B & 63] ? 2 : CmdTable[A & 63] < CmdTable[B & 63] ? 3 : 0; })
CMD(12, { if (A >= 64 || B > 64 - A) return 1; for (u32 i = 0; i < B; i++) CmdTable[A + i] = C; return 0; })
CMD(13, { u32 N = 0; for (u32 i = 0; i < 64; i++) N += CmdTable[i] == (u64)(B | C << 8); CmdTable[A & 63] = N; return 0; })
CMD(14, { CmdTable[A & 63] = ~CmdTable[B & 63]; return 0; })
CMD(15, { CmdTable[A & 63] &= CmdTable[B & 63] | C; return 0; })
CMD(16, { if (A >= 64) return 1; u64 V = CmdTable[A], R = 0; while (V) { R += V & 1; V >>= 1; } CmdTable[B & 63] = R; return 0; })
CMD(17, { if (A >= 64 || B >= 64) return 1; CmdTable[A] = CmdTable[A] > CmdTable[B] ? CmdTable[A] - CmdTable[B] : CmdTable[B] - CmdTable[A]; return 0; })
CMD(18, { u64 H = 0xCBF29CE484222325ull; for (u32 i = 0; i < (A & 63); i++) H = (H ^ CmdTable[i]) * 0x100000001B3ull; CmdTable[B & 63] = H; return 0; })
CMD(19, { if (C > 63) return 1; CmdTable[A & 63] = (CmdTable[A & 63] >> C) & ((1ull << (B & 63)) - 1); return 0; })
CMD(20, { if (A >= 64 || B >= 64 || A > B) return 1; for (u32 i = A, j = B; i < j; i++, j--) { u64 T = CmdTable[i]; CmdTable[i] = CmdTable[j]; CmdTable[j] = T; } return 0; })
CMD(21, { u32 Best = 0; for (u32 i = 1; i < 64; i++) if (CmdTable[i] > CmdTable[Best]) Best = i; return Best == (A & 63) ? 2 : 0; })
CMD(22, { if (!C) return 1; CmdTable[A & 63] = CmdTable[B & 63] * C / (C + 1); return 0; })
CMD(23, { u64 V = CmdTable[A & 63]; u32 D = 0; do { D++; V /= 10; } while (V); CmdTable[B & 63] = D; return 0; })
CMD(24, { if (A >= 64 || B > 64 - A || C >= 64) return 1; u64 S = 0; for (u32 i = 0; i < B; i++) S ^= CmdTable[A + i] << (i & 7); CmdTable[C] = S; return 0; })
CMD(25, { if (A >= 64) return 1; CmdTable[A] = CmdTable[A] ? 63 - __builtin_clzll(CmdTable[A]) : 64; return 0; })
CMD(26, { if (B >= 8) return 1; CmdTable[A & 63] |= (u64)C << (8 * B); return 0; })
CMD(27, { if (A >= 64 || B >= 64) return 1; return CmdTable[A] == CmdTable[B] ? 2 : CmdTable[A] & CmdTable[B] ? 3 : 0; })
CMD(28, { u32 N = 0; for (u32 i = 0; i < 64; i++) if ((CmdTable[i] & 0xff) == A) N++; CmdTable[B & 63] = N; return N > C ? 2 : 0; })
CMD(29, { if (A >= 64) return 1; CmdTable[A] = (CmdTable[A] * 6364136223846793005ull + 1442695040888963407ull) >> (C & 31); return 0; })
CMD(30, { for (u32 i = 0; i < 64; i++) CmdTable[i] = (CmdTable[i] + A) ^ B; return 0; })
CMD(31, { if (A >= 64 || B >= 64 || C >= 64) return 1; CmdTable[C] = CmdTable[A] < CmdTable[B] ? CmdTable[A] : CmdTable[B]; return 0; })
static const CmdFn CmdFns[32] = {Cmd0, Cmd1, Cmd2, Cmd3, Cmd4, Cmd5, Cmd6, Cmd7, Cmd8, Cmd9, Cmd10,
                                 Cmd11, Cmd12, Cmd13, Cmd14, Cmd15, Cmd16, Cmd17, Cmd18, Cmd19, Cmd20, Cmd21,
                                 Cmd22, Cmd23, Cmd24, Cmd25, Cmd26, Cmd27, Cmd28, Cmd29, Cmd30, Cmd31};
__attribute__((noipa)) static u32 TriggerCommands(const u8 *User, u64 Size) {
  u8 Kernel[256];
  if (Size > sizeof(Kernel) || (Size & 3)) return STATUS_INVALID_PARAMETER;
  KTRY T;
  TRY(T) {
    ProbeForRead(User, Size, 4);
    memcpy(Kernel, User, Size);
    END_TRY();
  }
  EXCEPT {
    END_TRY();
    return STATUS_ACCESS_VIOLATION;
  }
  u64 Acc = 0;
  for (u64 i = 0; i < Size; i += 4) {
    const u8 Op = Kernel[i];
    if (Op >= 32) return STATUS_INVALID_PARAMETER;
    const u32 R = CmdFns[Op](Kernel[i + 1], Kernel[i + 2], Kernel[i + 3]);
    if (R == 1) return STATUS_INVALID_PARAMETER;
    Acc = Acc * 3 + R;
  }
  LastInformation = Acc;
  return STATUS_SUCCESS;
}

/* the secure form of TriggerBufferOverflowStack: the copy is bounded */
__attribute__((noipa)) static u32 TriggerSecureCopy(const u8 *User, u64 Size) {
  u8 Kernel[512];
  KTRY T;
  memset(Kernel, 0, sizeof(Kernel));
  TRY(T) {
    ProbeForRead(User, sizeof(Kernel), 1);
    memcpy(Kernel, User, Size < sizeof(Kernel) ? Size : sizeof(Kernel));
    END_TRY();
  }
  EXCEPT {
    END_TRY();
    return STATUS_ACCESS_VIOLATION;
  }
  LastInformation = Size < sizeof(Kernel) ? Size : sizeof(Kernel);
  return Kernel[0] ? STATUS_SUCCESS : STATUS_UNSUCCESSFUL;
}
#endif

/* ---- dispatch (NtDeviceIoControlFile -> IrpDeviceIoCtlHandler) */
#ifdef HEVD_IO
__attribute__((noipa)) static u32 HevdDispatchIoctl(u32 Code, const u8 *User, u64 Size) {
#else
__attribute__((noipa, used)) u64 NtDeviceIoControlFile(u64 Handle, u32 Code, const u8 *User, u64 Size) {
  (void)Handle;
#endif
  u32 Status;
  DbgPrintEx(77, 3, "****** HEVD_IOCTL 0x%x ******\n", Code);
  switch (Code) {
    case 0x222003: Status = TriggerBufferOverflowStack(User, Size); break;
    case 0x222007: Status = TriggerBufferOverflowStackGS(User, Size); break;
    case 0x22200B: Status = TriggerArbitraryWrite(User, Size); break;
    case 0x22200F: Status = TriggerPoolOverflow(User, Size); break;
    case 0x222013: Status = TriggerNullPointerDereference(User, Size); break;
    case 0x222017: Status = TriggerIntegerOverflow(User, Size); break;
    case 0x22201B: Status = TriggerTypeConfusion(User, Size); break;
    case 0x22201F: Status = TriggerWait(User, Size); break;
#ifdef HEVD_IO
    case 0x222023: Status = TriggerChecksum(User, Size); break;
    case 0x222027: Status = TriggerParseRecords(User, Size); break;
    case 0x22202B: Status = TriggerSecureCopy(User, Size); break;
    case 0x22202F: Status = TriggerCommands(User, Size); break;
#endif
    default:
      DbgPrintEx(77, 3, "[-] Invalid IOCTL Code: 0x%X\n", Code);
      Status = STATUS_INVALID_DEVICE_REQUEST;
  }
  return Status;
}

#ifdef HEVD_IO
/* ---- the I/O manager (HEVD_IO) */
#define IRP_MJ_DEVICE_CONTROL 0x0e
#define IRP_MJ_MAXIMUM_FUNCTION 0x1b
#define IO_TYPE_DEVICE 3
#define IO_TYPE_DRIVER 4
#define IO_TYPE_FILE 5
#define IO_TYPE_IRP 6
#define STATUS_INVALID_HANDLE 0xC0000008u
#define STATUS_ACCESS_DENIED 0xC0000022u
#define STATUS_OBJECT_TYPE_MISMATCH 0xC0000024u
#define STATUS_INSUFFICIENT_RESOURCES 0xC000009Au
#define SL_INVOKE_ON_SUCCESS 0x40
#define SL_INVOKE_ON_ERROR 0x80
struct ListEntry {
  struct ListEntry *Flink, *Blink;
};
struct IoStatusBlock {
  u64 Status, Information;
};
struct DeviceObject;
struct Irp;
typedef u32 (*DriverDispatch)(struct DeviceObject *, struct Irp *);
typedef u32 (*IoCompletion)(struct DeviceObject *, struct Irp *, void *);
struct DriverObject {
  u16 Type, Size;
  u32 Flags;
  struct DeviceObject *DeviceObject;
  DriverDispatch MajorFunction[IRP_MJ_MAXIMUM_FUNCTION + 1];
};
struct DeviceObject {
  u16 Type, Size;
  u32 ReferenceCount;
  struct DriverObject *DriverObject;
  struct DeviceObject *LowerDevice; /* the filter's target (IoAttachDeviceToDeviceStack) */
  u32 Flags;
  u8 StackSize;
  u64 DeviceExtension[4];
};
struct FileObject {
  u16 Type, Size;
  struct DeviceObject *DeviceObject;
  u64 FinalStatus;
  u32 Flags;
  volatile u32 HandleCount, PointerCount;
};
struct HandleEntry {
  struct FileObject *Object;
  u32 GrantedAccess, Attributes;
};
struct IoStackLocation {
  u8 MajorFunction, MinorFunction, Flags, Control;
  u32 OutputBufferLength, InputBufferLength, Parameters_IoControlCode;
  const u8 *Type3InputBuffer;
  struct DeviceObject *DeviceObject;
  struct FileObject *FileObject;
  IoCompletion CompletionRoutine;
  void *Context;
};
#define IRP_STACK 4
struct Irp {
  u16 Type, Size;
  u32 Flags;
  struct Irp *NextFree; /* lookaside link */
  struct ListEntry ThreadListEntry;
  struct IoStatusBlock IoStatus;
  struct IoStatusBlock *UserIosb;
  void *UserBuffer;
  u8 StackCount, CurrentLocation, RequestorMode, PendingReturned;
  u32 Cancel;
  struct IoStackLocation *CurrentStackLocation;
  struct IoStackLocation Stack[IRP_STACK];
};
struct KEvent {
  u32 Type, SignalState;
  struct ListEntry WaitListHead;
};
struct KThread {
  struct ListEntry IrpList;
  u32 KernelApcDisable;
  u64 ContextSwitches;
};

static u32 HevdIrpDeviceIoCtlHandler(struct DeviceObject *Dev, struct Irp *Irp);
static u32 FilterDispatch(struct DeviceObject *Dev, struct Irp *Irp);
static u32 IopDefaultDispatch(struct DeviceObject *Dev, struct Irp *Irp);
static struct DriverObject HevdDriver, FilterDriver;
static struct DeviceObject HevdDevice = {IO_TYPE_DEVICE, sizeof(struct DeviceObject), 2, &HevdDriver, 0, 0, 1, {0}};
static struct DeviceObject FilterDevice = {IO_TYPE_DEVICE, sizeof(struct DeviceObject), 2, &FilterDriver, &HevdDevice,
                                           0, 2, {0}};
static struct FileObject HevdFile = {IO_TYPE_FILE, sizeof(struct FileObject), &FilterDevice, 0, 0, 1, 1};
static struct HandleEntry HandleTable[64];
static struct KThread CurrentThread;
static struct KEvent FileEvent;
static struct Irp IrpLookasideSlab[4];
static struct Irp *IrpLookaside;
static u32 IoInitialized;

/* the driver objects' tables as DriverEntry fills them (every major function
 * defaulted, then the ones the driver handles); the one-time setup a booted
 * system already did, redone here on the snapshot's first request only
 * because the synthetic image has no boot */
static void IopInitialize(void) {
  for (int i = 0; i <= IRP_MJ_MAXIMUM_FUNCTION; i++) {
    HevdDriver.MajorFunction[i] = IopDefaultDispatch;
    FilterDriver.MajorFunction[i] = FilterDispatch;
  }
  HevdDriver.Type = FilterDriver.Type = IO_TYPE_DRIVER;
  HevdDriver.MajorFunction[IRP_MJ_DEVICE_CONTROL] = HevdIrpDeviceIoCtlHandler;
  HevdDriver.DeviceObject = &HevdDevice;
  FilterDriver.DeviceObject = &FilterDevice;
  HandleTable[0x3C >> 2].Object = &HevdFile;
  HandleTable[0x3C >> 2].GrantedAccess = 0x0012019F; /* FILE_GENERIC_READ | FILE_GENERIC_WRITE */
  CurrentThread.IrpList.Flink = CurrentThread.IrpList.Blink = &CurrentThread.IrpList;
  FileEvent.WaitListHead.Flink = FileEvent.WaitListHead.Blink = &FileEvent.WaitListHead;
  for (int i = 0; i < 4; i++) {
    IrpLookasideSlab[i].NextFree = IrpLookaside;
    IrpLookaside = &IrpLookasideSlab[i];
  }
  IoInitialized = 1;
}

static void InsertTailList(struct ListEntry *Head, struct ListEntry *E) {
  E->Flink = Head;
  E->Blink = Head->Blink;
  Head->Blink->Flink = E;
  Head->Blink = E;
}
static void RemoveEntryList(struct ListEntry *E) {
  E->Blink->Flink = E->Flink;
  E->Flink->Blink = E->Blink;
}

__attribute__((noipa)) static u32 ObReferenceObjectByHandle(u64 Handle, u32 Access, struct FileObject **Out) {
  const u64 Index = Handle >> 2;
  if ((Handle & 3) || Index >= 64 || !HandleTable[Index].Object) return STATUS_INVALID_HANDLE;
  const struct HandleEntry *E = &HandleTable[Index];
  if ((E->GrantedAccess & Access) != Access) return STATUS_ACCESS_DENIED;
  if (E->Object->Type != IO_TYPE_FILE) return STATUS_OBJECT_TYPE_MISMATCH;
  __atomic_add_fetch(&E->Object->PointerCount, 1, __ATOMIC_SEQ_CST);
  *Out = E->Object;
  return STATUS_SUCCESS;
}
__attribute__((noipa)) static void ObDereferenceObject(struct FileObject *F) {
  __atomic_sub_fetch(&F->PointerCount, 1, __ATOMIC_SEQ_CST);
}

__attribute__((noipa)) static struct Irp *IoAllocateIrp(u8 StackSize) {
  struct Irp *Irp = IrpLookaside;
  if (Irp) IrpLookaside = Irp->NextFree;
  else Irp = ExAllocatePoolWithTag(0, sizeof(struct Irp), 0x20707249 /* 'Irp ' */);
  if (!Irp || StackSize > IRP_STACK) return 0;
  memset(Irp, 0, sizeof(*Irp));
  Irp->Type = IO_TYPE_IRP;
  Irp->Size = sizeof(*Irp);
  Irp->StackCount = StackSize;
  Irp->CurrentLocation = StackSize + 1;
  Irp->CurrentStackLocation = &Irp->Stack[StackSize];
  Irp->ThreadListEntry.Flink = Irp->ThreadListEntry.Blink = &Irp->ThreadListEntry;
  return Irp;
}
static void IoFreeIrp(struct Irp *Irp) {
  if (Irp >= IrpLookasideSlab && Irp < IrpLookasideSlab + 4) {
    Irp->NextFree = IrpLookaside;
    IrpLookaside = Irp;
  } else {
    ExFreePoolWithTag(Irp, 0x20707249);
  }
}
static struct IoStackLocation *IoGetNextIrpStackLocation(struct Irp *Irp) { return Irp->CurrentStackLocation - 1; }

__attribute__((noipa)) static u32 IofCallDriver(struct DeviceObject *Dev, struct Irp *Irp) {
  Irp->CurrentLocation--;
  if (!Irp->CurrentLocation) KeBugCheckEx(0x35, (u64)Irp, 0, 0, 0); /* NO_MORE_IRP_STACK_LOCATIONS */
  struct IoStackLocation *Sp = --Irp->CurrentStackLocation;
  Sp->DeviceObject = Dev;
  return Dev->DriverObject->MajorFunction[Sp->MajorFunction](Dev, Irp);
}

static void KeSetEvent(struct KEvent *E) {
  E->SignalState = 1;
  if (E->WaitListHead.Flink != &E->WaitListHead) ((void (*)(void))SwapContext)(); /* a waiter runs */
}

/* the thread's kernel APC queue: IofCompleteRequest's second stage runs as a
 * special kernel APC in the requesting thread (KeInsertQueueApc, delivered by
 * KiDeliverApc when the IRQL drops) */
struct KApc {
  struct ListEntry Entry;
  void (*Routine)(struct KApc *);
  void *Arg;
  u32 Inserted;
};
static struct ListEntry ApcListHead = {&ApcListHead, &ApcListHead};
static u32 ApcPending;
static void KeInsertQueueApc(struct KApc *A) {
  if (A->Inserted) return;
  A->Inserted = 1;
  InsertTailList(&ApcListHead, &A->Entry);
  ApcPending = 1;
}
__attribute__((noipa)) static void KiDeliverApc(void) {
  while (ApcListHead.Flink != &ApcListHead) {
    struct ListEntry *E = ApcListHead.Flink;
    RemoveEntryList(E);
    struct KApc *A = (struct KApc *)E;
    A->Inserted = 0;
    A->Routine(A);
  }
  ApcPending = 0;
}
/* the second stage (IopCompleteRequest): the status block to the caller, the
 * event, the IRP off the thread's list and freed, the file object dereferenced */
static void IopCompleteRequest(struct KApc *A) {
  struct Irp *Irp = A->Arg;
  *Irp->UserIosb = Irp->IoStatus;
  KeSetEvent(&FileEvent);
  RemoveEntryList(&Irp->ThreadListEntry);
  CurrentThread.KernelApcDisable--;
  ObDereferenceObject(Irp->Stack[Irp->StackCount - 1].FileObject);
  IoFreeIrp(Irp);
}
static struct KApc CompletionApc;
/* completion routines from the current location up, then the APC */
__attribute__((noipa)) static void IofCompleteRequest(struct Irp *Irp) {
  while (Irp->CurrentLocation <= Irp->StackCount) {
    struct IoStackLocation *Sp = Irp->CurrentStackLocation;
    Irp->CurrentLocation++;
    Irp->CurrentStackLocation++;
    const u32 Ok = (u32)Irp->IoStatus.Status < 0x80000000u;
    if (Sp->CompletionRoutine && (Sp->Control & (Ok ? SL_INVOKE_ON_SUCCESS : SL_INVOKE_ON_ERROR)))
      Sp->CompletionRoutine(Irp->CurrentLocation <= Irp->StackCount ? Irp->CurrentStackLocation->DeviceObject : 0,
                            Irp, Sp->Context);
  }
  CompletionApc.Routine = IopCompleteRequest;
  CompletionApc.Arg = Irp;
  KeInsertQueueApc(&CompletionApc);
}

static u32 IopDefaultDispatch(struct DeviceObject *Dev, struct Irp *Irp) {
  (void)Dev;
  Irp->IoStatus.Status = STATUS_INVALID_DEVICE_REQUEST;
  IofCompleteRequest(Irp);
  return STATUS_INVALID_DEVICE_REQUEST;
}

/* a filter above HEVD: its stack location copied down, a completion routine
 * that accounts the result in the device extension */
static u32 FilterCompletion(struct DeviceObject *Dev, struct Irp *Irp, void *Context) {
  (void)Dev;
  struct DeviceObject *F = Context;
  F->DeviceExtension[0]++;
  F->DeviceExtension[1] += Irp->IoStatus.Information;
  if ((u32)Irp->IoStatus.Status >= 0x80000000u) F->DeviceExtension[2]++;
  return STATUS_SUCCESS;
}
static u32 FilterDispatch(struct DeviceObject *Dev, struct Irp *Irp) {
  struct IoStackLocation *Sp = Irp->CurrentStackLocation, *Next = IoGetNextIrpStackLocation(Irp);
  *Next = *Sp; /* IoCopyCurrentIrpStackLocationToNext */
  Next->CompletionRoutine = 0;
  Next->Control = 0;
  Sp->CompletionRoutine = FilterCompletion;
  Sp->Context = Dev;
  Sp->Control = SL_INVOKE_ON_SUCCESS | SL_INVOKE_ON_ERROR;
  Dev->DeviceExtension[3]++;
  return IofCallDriver(Dev->LowerDevice, Irp);
}

/* WPP-style request tracing: the IOCTL and a hex dump of the buffer's head go
 * into the driver's circular trace buffer (what a driver's WPP / ETW provider
 * does for every request, without DbgPrintEx) */
static struct {
  u64 Sequence;
  u32 Head;
  char Data[8192];
} TraceBuffer;
static void TracePut(char C) {
  TraceBuffer.Data[TraceBuffer.Head] = C;
  TraceBuffer.Head = (TraceBuffer.Head + 1) & 8191;
}
__attribute__((noipa)) static void WppTraceRequest(u32 Code, const u8 *User, u64 Size) {
  static const char Hex[] = "0123456789abcdef";
  TraceBuffer.Sequence++;
  for (int i = 28; i >= 0; i -= 4) TracePut(Hex[(Code >> i) & 15]);
  TracePut(' ');
  const u64 N = Size < 192 ? Size : 192;
  KTRY T;
  TRY(T) {
    ProbeForRead(User, N, 1);
    for (u64 i = 0; i < N; i++) {
      const u8 B = User[i];
      TracePut(Hex[B >> 4]);
      TracePut(Hex[B & 15]);
      if ((i & 15) == 15) TracePut('\n');
    }
    END_TRY();
  }
  EXCEPT {
    END_TRY();
    TracePut('!');
  }
  TracePut('\n');
}

/* HEVD's IRP_MJ_DEVICE_CONTROL handler: the request from its stack location */
static u32 HevdIrpDeviceIoCtlHandler(struct DeviceObject *Dev, struct Irp *Irp) {
  (void)Dev;
  struct IoStackLocation *Sp = Irp->CurrentStackLocation;
  LastInformation = 0;
  WppTraceRequest(Sp->Parameters_IoControlCode, Sp->Type3InputBuffer, Sp->InputBufferLength);
  const u32 Status = HevdDispatchIoctl(Sp->Parameters_IoControlCode, Sp->Type3InputBuffer, Sp->InputBufferLength);
  Irp->IoStatus.Status = Status;
  Irp->IoStatus.Information = LastInformation;
  IofCompleteRequest(Irp);
  return Status;
}

/* NtDeviceIoControlFile for a METHOD_NEITHER request */
__attribute__((noipa, used)) u64 NtDeviceIoControlFile(u64 Handle, u32 Code, const u8 *User, u64 Size) {
  if (!IoInitialized) IopInitialize();
  struct FileObject *File;
  u32 Status = ObReferenceObjectByHandle(Handle, (Code >> 14) & 3 ? 0x3 : 0, &File);
  if (Status) return Status;
  struct DeviceObject *Top = File->DeviceObject;
  struct Irp *Irp = IoAllocateIrp(Top->StackSize);
  if (!Irp) {
    ObDereferenceObject(File);
    return STATUS_INSUFFICIENT_RESOURCES;
  }
  struct IoStatusBlock Iosb = {0, 0};
  Irp->UserIosb = &Iosb;
  Irp->RequestorMode = 1; /* UserMode */
  Irp->UserBuffer = 0;
  FileEvent.SignalState = 0; /* KeClearEvent */
  CurrentThread.KernelApcDisable++;
  InsertTailList(&CurrentThread.IrpList, &Irp->ThreadListEntry);
  struct IoStackLocation *Sp = IoGetNextIrpStackLocation(Irp);
  Sp->MajorFunction = IRP_MJ_DEVICE_CONTROL;
  Sp->FileObject = File;
  Sp->Parameters_IoControlCode = Code;
  Sp->InputBufferLength = (u32)Size;
  Sp->OutputBufferLength = 0;
  Sp->Type3InputBuffer = User;
  Irp->Stack[Top->StackSize - 1].FileObject = File;
  IofCallDriver(Top, Irp);
  if (ApcPending) KiDeliverApc(); /* KeLowerIrql / KiCheckForKernelApcDelivery */
  return Iosb.Status;
}
#endif

/* ---- system-call entry (LSTAR): rcx = user rip, r11 = user rflags,
 * r10 / rdx / r8 / r9 = arguments. The per-processor block (gs after SWAPGS)
 * holds the user rsp save slot (+0x10) and the kernel stack top (+0x1a8). */
__asm__(".globl KiSystemCall64\n"
        ".p2align 4\n"
        "KiSystemCall64:\n"
        "  swapgs\n"
        "  mov %rsp, %gs:0x10\n"
        "  mov %gs:0x1a8, %rsp\n"
        "  push %rcx\n"
        "  push %r11\n"
#ifdef HEVD_IO
        /* KTRAP_FRAME: the volatile registers and the user rsp, restored on the way out */
        "  push %gs:0x10\n"
        "  push %rax\n  push %rdx\n  push %r8\n  push %r9\n  push %r10\n  push %rbp\n"
        "  mov %rsp, %rbp\n"
        /* the volatile XMM registers, as KiSystemCall64 saves them in KTRAP_FRAME */
        "  sub $0x68, %rsp\n"
        "  movdqu %xmm0, 0x00(%rsp)\n  movdqu %xmm1, 0x10(%rsp)\n  movdqu %xmm2, 0x20(%rsp)\n"
        "  movdqu %xmm3, 0x30(%rsp)\n  movdqu %xmm4, 0x40(%rsp)\n  movdqu %xmm5, 0x50(%rsp)\n"
        "  sub $0x20, %rsp\n"        /* home space; rsp = 8 mod 16 at the callee's entry */
        "  mov %r10, %rcx\n"
        "  call NtDeviceIoControlFile\n"
        "  movdqu 0x20(%rsp), %xmm0\n  movdqu 0x30(%rsp), %xmm1\n  movdqu 0x40(%rsp), %xmm2\n"
        "  movdqu 0x50(%rsp), %xmm3\n  movdqu 0x60(%rsp), %xmm4\n  movdqu 0x70(%rsp), %xmm5\n"
        "  mov %rbp, %rsp\n"
        "  pop %rbp\n  pop %r10\n  pop %r9\n  pop %r8\n  pop %rdx\n"
        "  add $16, %rsp\n"          /* rax (the status is the return value) and the saved rsp slot */
#else
        "  sub $0x20, %rsp\n"        /* home space; rsp = 8 mod 16 at the callee's entry */
        "  mov %r10, %rcx\n"
        "  call NtDeviceIoControlFile\n"
        "  add $0x20, %rsp\n"
#endif
        "  pop %r11\n"
        "  pop %rcx\n"
        "  mov %gs:0x10, %rsp\n"
        "  swapgs\n"
        "  sysretq\n");

/* ---- exception entry (the IDT built by hevd.py points here). A kernel-mode
 * fault bugchecks the way Windows reports it: #PF as
 * PAGE_FAULT_IN_NONPAGED_AREA(cr2, access, rip, 0), the others as
 * KMODE_EXCEPTION_NOT_HANDLED(NTSTATUS, rip, 0, 0). A user-mode fault ends the
 * thread: the scheduler switches away (nt!SwapContext). */
struct TrapFrame {
  u64 Error, Rip, Cs, Rflags, Rsp, Ss;
};
__attribute__((noipa, used)) u32 KiTrapHandler(u64 Vector, struct TrapFrame *F, u64 Cr2) {
  if (F->Cs & 3) ((void (*)(void))SwapContext)();
  if (Vector == 14 && CurrentTry && Cr2 < 0x800000000000ull) {
    F->Rip = (u64)KiTryResume; /* dispatched to the guarded region's handler */
    return 1;
  }
  if (Vector == 14)
    KeBugCheckEx(0x50, Cr2, (F->Error & 0x10) ? 0x10 : (F->Error & 2) ? 2 : 0, F->Rip, 0);
  KeBugCheckEx(0x1E, Vector == 0 ? 0xC0000094u : Vector == 6 ? 0xC000001Du : 0xC0000005u, F->Rip, 0, 0);
  return 0;
}
/* stubs: faults without an error code push a zero so every frame is a TrapFrame */
__asm__(".globl KiDivideErrorFault\n.globl KiInvalidOpcodeFault\n.globl KiGeneralProtectionFault\n"
        ".globl KiPageFault\n"
        ".p2align 4\nKiDivideErrorFault:\n  push $0\n  mov $0, %ecx\n  jmp KiTrapCommon\n"
        ".p2align 4\nKiInvalidOpcodeFault:\n  push $0\n  mov $6, %ecx\n  jmp KiTrapCommon\n"
        ".p2align 4\nKiGeneralProtectionFault:\n  mov $13, %ecx\n  jmp KiTrapCommon\n"
        ".p2align 4\nKiPageFault:\n  mov $14, %ecx\n  jmp KiTrapCommon\n"
        "KiTrapCommon:\n"
        "  mov %rsp, %rdx\n"
        "  mov %cr2, %r8\n"
        "  and $-16, %rsp\n"
        "  push %rdx\n"
        "  push %rdx\n"
        "  sub $0x20, %rsp\n"
        "  call KiTrapHandler\n"
        "  add $0x28, %rsp\n"
        "  pop %rsp\n"          /* the trap frame */
        "  test %eax, %eax\n"
        "  jz 1f\n"
        "  add $8, %rsp\n"      /* error code */
        "  iretq\n"
        "1: hlt\n");
