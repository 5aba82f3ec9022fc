// Test infrastructure (tests/test_lane_host.py): the product's lane tokenizer
// logic -- lddl_amd/csrc/tokenize_lane.h, the per-lane walk that
// tokenize_lane.hip runs as waves on the GPU -- built for the host with g++
// under AddressSanitizer + UBSan.  A wave of 64 lanes is emulated lane by
// lane with the device kernel's wave-level steps (tile hand-out by batches,
// ring refills every REFILL_EVERY iterations, the batched slow pass), over
// the tables lddl_amd/csrc/tok_tables.h builds for the device.  Writes the
// staged ids (int32, by byte offset) and the counts, as host_serial.cpp does;
// tiles a lane gives up on are re-run by the serial path (tokenize_serial.h),
// as the device's fallback kernel does.
//   host_lane VOCAB TABLE BYTES OFFS N_SENT MAX_TOK OUT_IDS OUT_NTOK [SEG_TILES]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "tok_tables.h"
#include "tokenize_lane.h"
#include "tokenize_serial.h"

using namespace lddl;
using namespace lddl::tok6;

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

struct HostEnv {
  const TokParams& P;
  const LaneParams& Q;
  uint8_t* ring;  // this lane's RING_BYTES
  const uint16_t* ct;
  const uint32_t* asct;
  std::vector<int64_t>* aborted;
  uint32_t rbyte(int32_t q) const { return ring[((q >> 4) & (RING_SLOTS - 1)) * 16 + (q & 15)]; }
  uint32_t ctab(uint32_t b) const { return ct[b]; }
  uint2 trie(uint32_t i) const { return Q.trie[i]; }
  uint32_t bget(int i) const { return rbyte(i); }
  void bput(int i, uint32_t v) const { ring[((i >> 4) & (RING_SLOTS - 1)) * 16 + (i & 15)] = (uint8_t)v; }
  uint32_t raw(int64_t a) const { return P.bytes[a]; }
  uint32_t asc(uint32_t b) const { return asct[b]; }
  void put_tok(int64_t i, uint32_t id) const { Q.stage[i] = (uint16_t)id; }
  int64_t soff(int64_t i) const { return P.sent_off[i]; }
  void put_ntok(int64_t s, int32_t n, uint32_t) const { P.out_ntok[s] = n; }
  void abort_tile(const LaneState& L) const { aborted->push_back(L.t); }
};

int main(int argc, char** argv) {
  if (argc != 9 && argc != 10) {
    fprintf(stderr, "usage: host_lane VOCAB TABLE BYTES OFFS N MAXTOK IDS NTOK [SEG_TILES]\n");
    return 2;
  }
  VocabTables V;
  UniTables T;
  std::string err;
  if (build_vocab_tables(argv[1], V, err) || build_uni_tables(argv[2], T, err)) {
    fprintf(stderr, "%s\n", err.c_str());
    return 2;
  }
  if (V.trie.empty() || !T.lane_ok) {
    fprintf(stderr, "tables not modelled by the lane tokenizer\n");
    return 3;
  }
  std::vector<uint8_t> bytes, offb;
  const int64_t n = atoll(argv[5]);
  const int max_tok = atoi(argv[6]);
  if (!slurp(argv[3], bytes) || !slurp(argv[4], offb) || offb.size() != (size_t)(n + 1) * 8) {
    fprintf(stderr, "bad input files\n");
    return 2;
  }
  bytes.resize(bytes.size() + 16, 0);  // (ring loads are 16-B granules)
  std::vector<int64_t> off((size_t)n + 1);
  memcpy(off.data(), offb.data(), offb.size());
  const int64_t base = off[0], span = off[n] - base;
  const int64_t n_tiles = (span >> 10) + 1;
  std::vector<int64_t> tile_sent((size_t)n_tiles + 1), tile_off((size_t)n_tiles + 1);
  for (int64_t t = 0, s = 0; t <= n_tiles; ++t) {  // as tile_bounds_kernel: first sentence starting at >= t KiB
    while (s < n && off[s] - base < (t << 10)) ++s;
    tile_sent[t] = t == n_tiles ? n : s;
    tile_off[t] = off[tile_sent[t]];
  }
  std::vector<uint16_t> stage((size_t)(span + max_tok + 64), 0);
  std::vector<int32_t> ntok((size_t)n, 0);

  TokParams P{};
  P.bytes = bytes.data();
  P.sent_off = off.data();
  P.n_sent = n;
  P.max_tok = max_tok;
  P.out_ntok = ntok.data();
  P.top = T.top.data();
  P.pages = T.pages.data();
  P.multi = reinterpret_cast<const uint4*>(T.multi.data());
  P.bmp = T.bmp.data();
  for (int k = 0; k < 5; ++k) P.special[k] = V.special[k];
  P.unk = V.special[1];
  P.slots = V.slots.data();
  P.bloom = V.bloom.data();
  P.slot_mask = V.slot_mask;
  P.pool = V.pool.data();
  P.voff = V.voff.data();
  P.maxb[0] = V.maxb[0];
  P.maxb[1] = V.maxb[1];
  uint32_t asct[128];
  for (uint32_t b = 0; b < 128; ++b) asct[b] = T.pages[(size_t)T.top[0] * 256 + b];

  const int64_t seg = argc == 10 ? atoll(argv[9]) : (int64_t)1 << 22;
  std::vector<int64_t> aborted;
  uint64_t iters = 0, busy = 0;
  for (int64_t t0 = 0; t0 < n_tiles; t0 += seg) {
    LaneParams Q{};
    Q.trie = V.trie.data();
    Q.rbase[0] = V.trie_base[0];
    Q.rbase[1] = V.trie_base[1];
    Q.segb = base + (t0 << 10);
    Q.stage = stage.data() + (t0 << 10);
    Q.bytes_end = off[n];
    Q.tile_sent = tile_sent.data();
    Q.tile_off = tile_off.data();
    Q.t0 = t0;
    Q.t1 = std::min(n_tiles, t0 + seg);
    // waves take batches in turn (one emulated wave after another: the
    // counter order differs from the device's, the result may not)
    int64_t ctr = 0;
    for (int wave = 0;; ++wave) {
      if (Q.t0 + ctr * LANE_BATCH >= Q.t1) break;
      std::vector<LaneState> L(64);
      std::vector<uint8_t> rings(64 * RING_BYTES, 0xEE);
      for (auto& l : L) l = LaneState{}, l.mode = M_NEED;
      int64_t bnext = 0, bend = 0;
      bool exhausted = false;
      uint32_t iter = 0, slow_age = 0;
      int64_t nbat = ctr++;
      for (;;) {
        auto ballot = [&](auto f) {
          uint64_t m = 0;
          for (int i = 0; i < 64; ++i)
            if (f(L[i])) m |= 1ull << i;
          return m;
        };
        if ((iter & (REFILL_EVERY - 1)) == 0) {
          for (int i = 0; i < 64; ++i) {
            LaneState& l = L[i];
            const bool act = l.mode == M_SCAN || l.mode == M_WORD || l.mode == M_SKIP;
            if (!act) continue;
            const int32_t keep = (l.mode == M_WORD && l.la >= 0) ? l.la : l.p;
            if ((keep >> 4) > l.rlo) l.rlo = keep >> 4;
            if (l.rhi < l.rlo) l.rhi = l.rlo;
            while (l.rhi - l.rlo < RING_SLOTS && l.tb16 + 16 * (int64_t)l.rhi < Q.bytes_end) {
              memcpy(&rings[i * RING_BYTES + (l.rhi & (RING_SLOTS - 1)) * 16], &bytes[l.tb16 + 16 * (int64_t)l.rhi], 16);
              ++l.rhi;
            }
          }
        }
        const uint64_t sw = ballot([](const LaneState& l) { return l.mode == M_SLOW; });
        if (sw) {
          ++slow_age;
          const uint64_t other = ballot([](const LaneState& l) { return l.mode >= M_TILE && l.mode != M_SLOW; });
          if (__builtin_popcountll(sw) >= SLOW_BATCH || slow_age >= SLOW_AGE || other == 0) {
            for (int i = 0; i < 64; ++i) {
              if (L[i].mode != M_SLOW) continue;
              const HostEnv en{P, Q, &rings[i * RING_BYTES], T.lane_ctab.data(), asct, &aborted};
              lane_slow(L[i], en);
            }
            slow_age = 0;
          }
        }
        busy += __builtin_popcountll(ballot([](const LaneState& l) { return l.mode >= M_TILE && l.mode != M_SLOW; }));
        for (int i = 0; i < 64; ++i) {
          const HostEnv en{P, Q, &rings[i * RING_BYTES], T.lane_ctab.data(), asct, &aborted};
          lane_step(L[i], en);
        }
        const uint64_t need = ballot([](const LaneState& l) { return l.mode == M_NEED; });
        if (need) {
          if (bnext >= bend && !exhausted) {
            const int64_t b = Q.t0 + nbat * LANE_BATCH;
            if (b < Q.t1) {
              bnext = b;
              bend = std::min(b + (int64_t)LANE_BATCH, Q.t1);
              nbat = ctr++;
            } else {
              exhausted = true;
            }
          }
          int k = 0;
          for (int i = 0; i < 64; ++i) {
            if (L[i].mode != M_NEED) continue;
            const int64_t t = bnext + k++;
            if (t < bend) {
              L[i].t = t;
              L[i].s = tile_sent[t];
              L[i].sb = tile_sent[t + 1];
              L[i].obase = tile_off[t];
              L[i].mode = M_TILE;
            } else if (exhausted) {
              L[i].mode = M_IDLE;
            }
          }
          bnext = std::min(bnext + (int64_t)__builtin_popcountll(need), bend);
        }
        ++iter;
        if (ballot([](const LaneState& l) { return l.mode != M_IDLE; }) == 0) break;
        if (iter > 400000000u) {
          fprintf(stderr, "wave %d does not finish\n", wave);
          return 4;
        }
      }
      iters += iter;
    }
  }
  // the serial path over the tiles given up on (the device's fallback kernel)
  if (!aborted.empty()) {
    std::vector<uint8_t> wbuf(WB_LDS + WB_OVF, 0);
    const GlobalWordBuf wb{wbuf.data()};
    TokParams F = P;
    F.out_ids = stage.data();
    uint32_t ascii_tab[128];
    for (uint32_t b = 0; b < 128; ++b) ascii_tab[b] = asct[b];
    for (int64_t t : aborted)
      for (int64_t s = tile_sent[t]; s < tile_sent[t + 1]; ++s) {
        SentState st{off[s], off[s + 1], off[s] - base, 0};
        while (st.p < st.e && st.ntok < P.max_tok) step(F, st, wb, ascii_tab);
        ntok[s] = st.ntok < max_tok ? st.ntok : max_tok;
      }
  }
  fprintf(stderr, "lane: waves' iterations %llu (bytes %lld), lane-iterations busy %.3f, tiles to the serial path %zu\n",
          (unsigned long long)iters, (long long)span, iters ? (double)busy / (64.0 * iters) : 0.0, aborted.size());
  FILE* fi = fopen(argv[7], "wb");
  FILE* fn = fopen(argv[8], "wb");
  if (!fi || !fn) return 2;
  std::vector<int32_t> ids32(stage.begin(), stage.begin() + (span > 0 ? span : 0));
  fwrite(ids32.data(), sizeof(int32_t), ids32.size(), fi);
  fwrite(ntok.data(), sizeof(int32_t), ntok.size(), fn);
  fclose(fi);
  fclose(fn);
  return 0;
}
