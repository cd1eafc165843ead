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

struct GsFrame {
  u8 Kernel[512];
  u64 Cookie;
};
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

/* ---- dispatch (NtDeviceIoControlFile -> IrpDeviceIoCtlHandler) */
__attribute__((noipa, used)) u64 NtDeviceIoControlFile(u64 Handle, u32 Code, const u8 *User, u64 Size) {
  (void)Handle;
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
    default:
      DbgPrintEx(77, 3, "[-] Invalid IOCTL Code: 0x%X\n", Code);
      Status = STATUS_INVALID_DEVICE_REQUEST;
  }
  return Status;
}

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
        "  sub $0x20, %rsp\n"        /* home space; rsp = 8 mod 16 at the callee's entry */
        "  mov %r10, %rcx\n"
        "  call NtDeviceIoControlFile\n"
        "  add $0x20, %rsp\n"
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
