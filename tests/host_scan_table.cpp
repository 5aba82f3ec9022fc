// Test driver (tests/test_scan_table.py): the scan's whole-word table
// (lddl_amd/csrc/tok_tables.h build_vocab_tables) built on the host under
// ASan/UBSan, then every whole-word key of <= 24 bytes looked up as the
// scan looks it up (vhash, its two candidate slots, the slot compare):
// found, with the id the vocab dictionary gives it (the last duplicate);
// and no slot holds anything else.
//   host_scan_table VOCAB  -> "keys N slots S misses M wrong W extra X"
#include <stdio.h>
#include <string.h>

#include <map>
#include <string>

#include "common.h"
#include "tok_tables.h"

using namespace lddl;

int main(int argc, char** argv) {
  if (argc != 2) return 2;
  VocabTables V;
  std::string err;
  if (build_vocab_tables(argv[1], V, err, false) != 0) {
    fprintf(stderr, "%s\n", err.c_str());
    return 1;
  }
  std::map<std::string, uint32_t> dict;  // whole words of <= 24 bytes -> last id
  for (size_t i = 0; i < V.vocab.size(); ++i) {
    const std::string& w = V.vocab[i];
    if (w.empty() || (w.size() >= 2 && w[0] == '#' && w[1] == '#') || w.size() > 24) continue;
    dict[w] = (uint32_t)i;
  }
  const uint32_t m = V.st_mask;
  long misses = 0, wrong = 0, extra = 0;
  for (const auto& kv : dict) {
    uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    memcpy(d, kv.first.data(), kv.first.size());
    const uint32_t len = (uint32_t)kv.first.size();
    const uint32_t h = vhash(d, len, 0);
    const uint32_t want = (len << 16) | 0x80000000u;
    long found = -1;
    for (uint32_t p : {h & m, st_second(h) & m}) {
      const uint32_t* s = &V.st[(size_t)p * 8];
      bool eq = (s[6] & 0xFFFF0000u) == want;
      for (int q = 0; q < 6; ++q) eq = eq && s[q] == d[q];
      if (eq) {
        found = s[6] & 0xFFFFu;
        break;
      }
    }
    if (found < 0) ++misses;
    else if ((uint32_t)found != kv.second) ++wrong;
  }
  size_t used = 0;
  for (size_t p = 0; p <= m; ++p) {
    const uint32_t* s = &V.st[p * 8];
    if (s[6] == 0) continue;
    ++used;
    const uint32_t len = (s[6] >> 16) & 0xFFu;
    std::string k(reinterpret_cast<const char*>(s), len);
    if (((s[6] >> 24) & 1u) || !dict.count(k)) ++extra;
  }
  printf("keys %zu slots %u used %zu misses %ld wrong %ld extra %ld\n", dict.size(), m + 1, used, misses, wrong, extra);
  return 0;
}
