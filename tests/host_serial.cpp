// Test infrastructure (tests/test_serial_host.py): the product's serial
// tokenizer path -- lddl_amd/csrc/tokenize_serial.h, the exact fallback of the
// split tokenizer (tokenize_fallback_kernel) -- built for the host with g++
// under AddressSanitizer + UBSan over the tables lddl_amd/csrc/tok_tables.h
// builds for the device.  Tokenises the sentences of a raw file (bytes +
// int64 offsets) at max_tok and writes the ids sparse by byte offset (int32)
// and the counts, as oracle/asan_driver.c does for the C restatement.
//   host_serial VOCAB TABLE BYTES OFFS N_SENT MAX_TOK OUT_IDS OUT_NTOK
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "tok_tables.h"
#include "tokenize_serial.h"

using namespace lddl;

static bool slurp(const char* path, std::vector<uint8_t>& out) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  fseek(f, 0, SEEK_END);
  const long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  out.resize(n > 0 ? (size_t)n : 0);
  const bool ok = n <= 0 || fread(out.data(), 1, (size_t)n, f) == (size_t)n;
  fclose(f);
  return ok;
}

int main(int argc, char** argv) {
  if (argc != 9) {
    fprintf(stderr, "usage: host_serial VOCAB TABLE BYTES OFFS N MAXTOK IDS NTOK\n");
    return 2;
  }
  VocabTables V;
  UniTables T;
  std::string err;
  if (build_vocab_tables(argv[1], V, err) || build_uni_tables(argv[2], T, err)) {
    fprintf(stderr, "%s\n", err.c_str());
    return 2;
  }
  std::vector<uint8_t> bytes, offb;
  const int64_t n = atoll(argv[5]);
  const int max_tok = atoi(argv[6]);
  if (!slurp(argv[3], bytes) || !slurp(argv[4], offb) || offb.size() != (size_t)(n + 1) * 8) {
    fprintf(stderr, "bad input files\n");
    return 2;
  }
  std::vector<int64_t> off((size_t)n + 1);
  memcpy(off.data(), offb.data(), offb.size());
  const int64_t base = off[0], span = off[n] - base;
  std::vector<uint16_t> ids(span > 0 ? (size_t)span : 1, 0);
  std::vector<int32_t> ntok((size_t)n, 0);

  TokParams P{};
  P.bytes = bytes.data();
  P.sent_off = off.data();
  P.n_sent = n;
  P.max_tok = max_tok;
  P.out_ids = ids.data();
  P.top = T.top.data();
  P.pages = T.pages.data();
  P.multi = reinterpret_cast<const uint4*>(T.multi.data());
  P.bmp = T.bmp.data();
  P.xmap = T.xmap.data();
  P.slots = V.slots.data();
  P.bloom = V.bloom.data();
  P.slot_mask = V.slot_mask;
  P.pool = V.pool.data();
  P.voff = V.voff.data();
  P.maxb[0] = V.maxb[0];
  P.maxb[1] = V.maxb[1];
  for (int k = 0; k < 5; ++k) P.special[k] = V.special[k];
  P.unk = V.special[1];
  P.vt = reinterpret_cast<const uint4*>(V.vt.data());
  P.vt_mask = V.vt_mask;
  P.vbloom = V.vbloom.data();

  uint32_t ascii_tab[128];
  for (uint32_t b = 0; b < 128; ++b) ascii_tab[b] = T.pages[(size_t)T.top[0] * 256 + b];
  std::vector<uint8_t> wbuf(WB_LDS + WB_OVF, 0);
  const GlobalWordBuf wb{wbuf.data()};
  for (int64_t s = 0; s < n; ++s) {
    SentState st{off[s], off[s + 1], off[s] - base, 0};
    while (st.p < st.e && st.ntok < P.max_tok) step(P, st, wb, ascii_tab);
    ntok[s] = st.ntok < max_tok ? st.ntok : max_tok;
  }

  FILE* fi = fopen(argv[7], "wb");
  FILE* fn = fopen(argv[8], "wb");
  if (!fi || !fn) return 2;
  std::vector<int32_t> ids32(ids.begin(), ids.begin() + (span > 0 ? span : 0));
  fwrite(ids32.data(), sizeof(int32_t), ids32.size(), fi);
  fwrite(ntok.data(), sizeof(int32_t), ntok.size(), fn);
  fclose(fi);
  fclose(fn);
  return 0;
}
