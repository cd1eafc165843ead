/* tlv_server guest — the program the synthetic tlv_server snapshot runs.
 *
 * A freestanding restatement of the packet handler of the reference target
 * (src/tlv_server/tlv_server.cc:14-94): a 4-entry chunk table driven by
 * Allocate / Edit / Delete packets of the form {u32 Command, u16 Id,
 * u16 BodySize, u8 Body[]}, with the same bugs (Allocate into a full table
 * writes one entry past the table; Allocate and Edit copy BodySize bytes from
 * a packet that may be shorter; Edit copies BodySize bytes into a chunk
 * allocated with a smaller size).
 *
 * It is compiled with gcc for x86-64 (-mabi=ms: Win64 argument registers, as
 * the module's handlers expect: rcx = packet, rdx = size, printf's format in
 * rcx) into a flat image placed in the snapshot by wtf_amd/tools/tlv.py.
 * The heap is a page heap: every allocation ends at the end of its own page,
 * followed by an unmapped guard page, so overflows fault like under a
 * page-heap-enabled Windows process; a bad free is a __fastfail: `int 0x29`
 * with the failure code in ecx, which the snapshot's IDT (gate 0x29, DPL 3)
 * delivers to nt!KiRaiseSecurityCheckFailure in ring 0 with the address after
 * the int at [rsp] (crash_detection_umode.cc:131-152).
 */
#include "sse_rt.h"
typedef unsigned long long u64;
typedef unsigned int u32;
typedef unsigned short u16;
typedef unsigned char u8;

#define HEAP_BASE 0x200000000ull
#define HEAP_SLOTS 64
#define HEAP_STRIDE 0x2000ull
#define PACKET_VA 0x300000000ull

enum { CmdAllocate = 0, CmdEdit = 1, CmdDelete = 2 };

struct Header {
  u32 Command;
  u16 Id;
  u16 BodySize;
};

struct Chunk {
  u16 Id;
  u16 Size;
  u8 *Buf;
};

/* One object so the layout is fixed: the entry past ChunkList is LastFreed,
 * a stale pointer to the buffer of the chunk deleted last (what a write past
 * the table lands on in this image): Allocate into a full table deletes it as
 * a Chunk, freeing whatever its bytes 8..15 hold, and the heap's free check
 * fails fast on a pointer it does not own. */
struct Globals {
  struct Chunk *ChunkList[4];
  struct Chunk *LastFreed;
  u64 FreeHead; /* 1 + index of the first free slot, 0 = none */
  u64 InUse;    /* bit per slot: allocated */
  u64 Initialised;
};
struct Globals G;

/* ---- stubs the snapshot exports as module symbols (breakpointed) */
__attribute__((noipa, used)) int printf(const char *Format, ...) {
  (void)Format;
  return 0;
}
__attribute__((noipa, used, naked)) void RtlDispatchException(void) { __asm__ volatile("hlt"); }
__attribute__((noipa, used, naked)) void KeBugCheck2(void) { __asm__ volatile("hlt"); }
__attribute__((noipa, used, naked)) void SwapContext(void) { __asm__ volatile("hlt"); }
__attribute__((noipa, used, naked)) void HalpPerfInterrupt(void) { __asm__ volatile("hlt"); }

/* ---- page heap */
static u8 *slot_page(u64 Slot) { return (u8 *)(HEAP_BASE + Slot * HEAP_STRIDE); }

static void heap_init(void) {
  /* free list threaded through the first 8 bytes of each slot page */
  for (u64 i = 0; i < HEAP_SLOTS; i++) *(u64 *)slot_page(i) = (i + 1 < HEAP_SLOTS) ? i + 2 : 0;
  G.FreeHead = 1;
  G.InUse = 0;
  G.Initialised = 1;
}

__attribute__((noinline)) static void *Malloc(u64 Size) {
  if (!G.Initialised) heap_init();
  if (G.FreeHead == 0 || Size > 0x1000) return 0;
  const u64 Slot = G.FreeHead - 1;
  u8 *Page = slot_page(Slot);
  G.FreeHead = *(u64 *)Page;
  G.InUse |= 1ull << Slot;
  *(u64 *)Page = 0;
  u8 *P = (u8 *)(((u64)Page + 0x1000 - Size) & ~7ull);
  sse_fill(P, 0, Size);
  return P;
}

__attribute__((noinline)) static void Free(void *P) {
  if (!P) return;
  const u64 Off = (u64)P - HEAP_BASE;
  if ((u64)P < HEAP_BASE || Off >= HEAP_SLOTS * HEAP_STRIDE || (Off & 0x1fff) >= 0x1000 ||
      !((G.InUse >> (Off / HEAP_STRIDE)) & 1)) {
    /* a block the heap does not own (a double free): __fastfail(FAST_FAIL_INVALID_FREE) */
    __asm__ volatile("mov $0x3e, %%ecx\n\tint $0x29" ::: "rcx", "memory");
    __builtin_unreachable();
  }
  G.InUse &= ~(1ull << (Off / HEAP_STRIDE));
  u8 *Page = slot_page(Off / HEAP_STRIDE);
  *(u64 *)Page = G.FreeHead;
  G.FreeHead = Off / HEAP_STRIDE + 1;
}

static void Memcpy(u8 *Dst, const u8 *Src, u64 Size) { sse_copy(Dst, Src, Size); }

static void DeleteChunk(struct Chunk *C) {
  if (!C) return;
  u8 *Buf = C->Buf;
  Free(Buf);
  Free(C);
  G.LastFreed = (struct Chunk *)Buf;
}

/* tlv_server.cc:31-94 */
__attribute__((noinline, used)) void ProcessPacket(const u8 *Packet, const u32 PacketSize) {
  const struct Header *Header = (const struct Header *)Packet;
  if (PacketSize < sizeof(*Header)) {
    printf("[!] Packet is not big enough to check the header\n");
    return;
  }
  const u32 Command = Header->Command;
  const u8 *Body = (const u8 *)(Header + 1);
  switch (Command) {
    case CmdAllocate: {
      printf("Allocate command\n");
      const u16 ChunkId = Header->Id;
      u64 Idx = 0;
      while (Idx < 4 && G.ChunkList[Idx] != 0) Idx++;
      struct Chunk *C = (struct Chunk *)Malloc(sizeof(struct Chunk));
      C->Id = ChunkId;
      C->Size = Header->BodySize;
      C->Buf = (u8 *)Malloc(C->Size);
      Memcpy(C->Buf, Body, C->Size);
      struct Chunk *Old = G.ChunkList[Idx]; /* Idx == 4: one past the table */
      G.ChunkList[Idx] = C;
      DeleteChunk(Old);
      break;
    }
    case CmdEdit: {
      printf("Edit command\n");
      const u16 ChunkId = Header->Id;
      u64 Idx = 0;
      while (Idx < 4 && !(G.ChunkList[Idx] != 0 && G.ChunkList[Idx]->Id == ChunkId)) Idx++;
      if (Idx == 4) {
        printf("[!] Couldn't find ChunkId 0x%x\n", ChunkId);
        return;
      }
      Memcpy(G.ChunkList[Idx]->Buf, Body, Header->BodySize);
      break;
    }
    case CmdDelete: {
      printf("Delete command\n");
      const u16 ChunkId = Header->Id;
      u64 Idx = 0;
      while (Idx < 4 && !(G.ChunkList[Idx] != 0 && G.ChunkList[Idx]->Id == ChunkId)) Idx++;
      if (Idx == 4) {
        printf("[!] Couldn't find ChunkId 0x%x\n", ChunkId);
        return;
      }
      struct Chunk *C = G.ChunkList[Idx];
      G.ChunkList[Idx] = 0;
      DeleteChunk(C);
      break;
    }
  }
}

/* The receive loop (tlv_server.cc:149-175): the snapshot is taken at the entry
 * of ProcessPacket called from here, so [rsp] = ServerLoopReturn. */
__attribute__((naked, used)) void ServerLoop(void) {
  __asm__ volatile(
      "1:\n"
      "  sub $40, %rsp\n"
      "  movabs $0x300000000, %rcx\n"
      "  mov $0x1000, %edx\n"
      "  call ProcessPacket\n"
      ".globl ServerLoopReturn\n"
      "ServerLoopReturn:\n"
      "  add $40, %rsp\n"
      "  jmp 1b\n");
}
