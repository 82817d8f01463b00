// DIAGNOSTIC (host): narde_rules.h select_bit (round 3: byte, then 4 / 2 / 1)
// against the round-2 12 / 6 / 3 / 1 / 1 search, for every 24-bit mask and
// every rank below its popcount.  Must print 0 mismatches.
//   hipcc -O2 -std=c++17 -o /tmp/select_check tools/diag/select_check.cpp && /tmp/select_check
#include <cstdio>

#include "../../gym-narde_amd/csrc/narde_rules.h"

static int select_round2(uint32_t m, int j) {
  int pos = 0;
  uint32_t c;
  c = __builtin_popcount(m & 0xFFFu);
  if ((uint32_t)j >= c) { j -= (int)c; m >>= 12; pos += 12; }
  c = __builtin_popcount(m & 0x3Fu);
  if ((uint32_t)j >= c) { j -= (int)c; m >>= 6; pos += 6; }
  c = __builtin_popcount(m & 0x7u);
  if ((uint32_t)j >= c) { j -= (int)c; m >>= 3; pos += 3; }
  c = m & 1u;
  if ((uint32_t)j >= c) { j -= (int)c; m >>= 1; pos += 1; }
  c = m & 1u;
  if ((uint32_t)j >= c) { pos += 1; }
  return pos;
}

int main() {
  long n = 0, bad = 0;
  for (uint32_t m = 0; m < (1u << 24); ++m) {
    const int c = __builtin_popcount(m);
    for (int j = 0; j < c; ++j) {
      ++n;
      bad += narde::select_bit(m, j) != select_round2(m, j);
    }
  }
  printf("checked %ld (mask, rank) pairs, mismatches %ld\n", n, bad);
  return bad != 0;
}
