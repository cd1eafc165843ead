/* hevd user guest — the ring-3 half of the synthetic HEVD snapshot: the
 * program the reference snapshot is taken in, stopped at its call to
 * DeviceIoControl (a 6-byte `call [rip+disp32]`, fuzzer_hevd.cc:66-67), and
 * the DeviceIoControl stub that enters the kernel with SYSCALL
 * (wtf_amd/tools/guest/hevd_kernel.c). */
typedef unsigned long long u64;

u64 (*pDeviceIoControl)(u64, u64, void *, u64, void *, u64, u64 *, void *);

/* kernelbase!DeviceIoControl -> ntdll!NtDeviceIoControlFile */
__asm__(".globl DeviceIoControl\n"
        ".p2align 4\n"
        "DeviceIoControl:\n"
        "  mov %rcx, %r10\n"
        "  mov $7, %eax\n"
        "  syscall\n"
        "  ret\n");

/* The snapshot's rip is CallSite with rcx..r9 and the stack arguments set up;
 * the module stops the testcase at CallSite + 6. */
__asm__(".globl UserMain\n"
        ".globl CallSite\n"
        ".p2align 4\n"
        "UserMain:\n"
        "  sub $0x48, %rsp\n"
        "CallSite:\n"
        "  call *pDeviceIoControl(%rip)\n"
        "  add $0x48, %rsp\n"
        "  hlt\n");
