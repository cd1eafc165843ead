// Reference checker driver (test infrastructure only): parses a kdmp file with
// the reference's own kdmp-parser headers (src/libs/kdmp-parser/src/lib,
// KernelDumpParser::Parse kdmp-parser.h:51-94, GetPhysicalPage :233-254,
// VirtTranslate :269-345) and prints what our restatement must reproduce:
//   "TYPE <dumptype>" "CR3 <dtb>" "RIP <rip>"
//   "PAGE <gpa> <fnv1a64 of the 4096 bytes>" for every physical page
//   "VT <gva> <gpa|-1>" for each gva given on the command line.
#include "kdmp-parser.h"
#include <cstdio>
#include <cstdlib>
#include <map>

static uint64_t fnv(const uint8_t *p, size_t n) {
  uint64_t h = 1469598103934665603ULL;
  for (size_t i = 0; i < n; i++) { h ^= p[i]; h *= 1099511628211ULL; }
  return h;
}

int main(int argc, char **argv) {
  if (argc < 2) { fprintf(stderr, "usage: kdmp_ref <dump> [gva...]\n"); return 2; }
  kdmpparser::KernelDumpParser P;
  if (!P.Parse(argv[1])) { printf("PARSE_FAIL\n"); return 1; }
  printf("TYPE %u\n", (unsigned)P.GetDumpType());
  printf("CR3 %llx\n", (unsigned long long)P.GetDirectoryTableBase());
  printf("RIP %llx\n", (unsigned long long)P.GetContext()->Rip);
  std::map<uint64_t, const uint8_t *> sorted(P.GetPhysmem().begin(), P.GetPhysmem().end());
  for (auto &[gpa, page] : sorted)
    printf("PAGE %llx %llx\n", (unsigned long long)gpa, (unsigned long long)fnv(page, 4096));
  for (int i = 2; i < argc; i++) {
    uint64_t gva = strtoull(argv[i], nullptr, 0);
    auto gpa = P.VirtTranslate(gva);
    if (gpa) printf("VT %llx %llx\n", (unsigned long long)gva, (unsigned long long)*gpa);
    else printf("VT %llx -1\n", (unsigned long long)gva);
  }
  return 0;
}
