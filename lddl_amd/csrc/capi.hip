// C-ABI of liblddl_amd.so: the drop-in boundary (declared in include/lddl_amd.h).
// Plain pointers and sizes only; device pointers come from the caller
// (torch tensors via data_ptr(), or hipMalloc).  Every entry point returns 0
// on success and a negative LDDL_E* code on failure; the message is kept in
// a thread-local buffer readable with lddl_last_error().  Nothing aborts.
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <string>
#include <vector>

#include "../../include/lddl_amd.h"
#include "tok_tables.h"
#include "collate.h"
#include "common.h"
#include "pack.h"
#include "render.h"
#include "tokenize.h"

using namespace lddl;

static thread_local char g_err[1024];

static int set_err(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess) return set_err(LDDL_EHIP, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

// a device buffer grown on demand
struct WsBuf {
  void* p = nullptr;
  size_t cap = 0;
};

// The result of one lddl_pack_* call, owned by the caller (lddl_pack_new):
// the pair records, their shuffled / binned order, the per-partition counts
// and offsets and (masking) the masked positions -- everything the post-pack
// calls (lddl_materialize, lddl_row_spans, lddl_masked_lm[_spans],
// lddl_row_docs) read.  A ctx holds one of its own for callers that pass
// NULL.  Buffers grow on demand and are reused by later packs into it.
struct lddl_pack {
  int device = 0;
  WsBuf ws[34];
  PackParams pp{};
  int64_t last_npairs = -1, last_ntok = -1, last_nmask = -1, last_nsent = 0, last_ndense = 0;
  int pack_codebert = 0;
  uint64_t mlm_cap = 0;  // masking arena capacity that last sufficed
  uint16_t* last_tokens = nullptr;  // rows of the last lddl_materialize of this result
  const int64_t* last_tok_off = nullptr;
  const int64_t* last_part = nullptr;
};

struct lddl_ctx {
  int device = 0;
  int n_cu = 0;
  int vocab_size = 0;
  uint32_t special[5] = {0, 0, 0, 0, 0};
  std::vector<std::string> vocab;  // host copy (for rendering / tests)
  // device tables
  uint16_t* d_top = nullptr;
  uint32_t* d_pages = nullptr;
  uint32_t* d_bmp = nullptr;  // flat entries of the Basic Multilingual Plane (top/pages resolved)
  uint32_t* d_xmap = nullptr;  // fast exception entries, one per code point (tokenize_split.hip XM_*)
  uint4* d_multi = nullptr;
  uint4* d_slots = nullptr;
  uint32_t* d_bloom = nullptr;
  uint32_t slot_mask = 0;
  uint8_t* d_pool = nullptr;
  uint32_t* d_voff = nullptr;
  uint8_t* d_rpool = nullptr;    // full vocab strings (incl. "##"), 4-aligned: rendering
  uint32_t* d_rinfo = nullptr;   // [V] offset << 8 | length into d_rpool
  uint32_t maxb[2] = {0, 0};
  uint4* d_vt = nullptr;         // v4 bucketed vocab table
  uint32_t vt_mask = 0;
  uint32_t* d_vbloom = nullptr;  // its Bloom filter
  uint4* d_st = nullptr;         // the scan's whole-word table
  uint32_t st_mask = 0;
  bool scan_ok = false;          // the ASCII page fits the split scan's per-byte class table
  // lane tokenizer (tokenize_lane.hip): the vocab trie, its roots, the byte classes
  uint2* d_trie = nullptr;
  uint32_t trie_base[2] = {0, 0};
  uint16_t* d_lane_ctab = nullptr;
  bool lane_ok = false;
  uint64_t* d_lane_stats = nullptr;
  // per-kernel timing of the split tokenizer (lddl_set_timing)
  bool timing = false;
  SplitTiming* tm = nullptr;
  unsigned long long* d_nrec = nullptr;
  int64_t last_tok_bytes = 0, last_tok_sent = 0;
  // per-sentence [CLS]/[SEP] flags written by the last lddl_tokenize (ws 41),
  // reused by a masked lddl_pack_bert over the same id / count buffers
  const void* spec_ids = nullptr;
  const void* spec_ntok = nullptr;
  const void* spec_soff = nullptr;
  int64_t spec_nsent = -1;
  bool spec_flags = false;  // lddl_set_special_flags
  // tokenizer / render / collate workspace (grown on demand)
  WsBuf ws[50];
  int64_t* h_tot = nullptr;  // pinned [8]
  lddl_pack own;             // the pack result of calls that pass no lddl_pack
  uint64_t mlm_cap0 = 0;     // initial masking arena (LDDL_MLM_CAP, tests)
  // scratch
  int tok_grid = 0;
  int tok_algo = 5;  // 5 = split tokenizer, 6 = lane tokenizer, 0 = every tile through the exact serial path
  uint8_t* d_ovf = nullptr;
  uint32_t* d_counter = nullptr;
  // debug counters of the tokenizer (LDDL_TOK_DEBUG=1) and of the packers
  // (LDDL_PACK_DEBUG=1: phase ticks + per-wave start / end), on this ctx's device
  uint64_t* d_tdbg = nullptr;
  uint64_t* d_pdbg = nullptr;
  int64_t pdbg_cap = 0;
  // collate: whole-token vocab table (built on first use)
  uint2* d_ctab = nullptr;
  uint32_t ctab_mask = 0;
};

// ------------------------------------------------------------------ pack --
template <class T>
static int ws_get(WsBuf* ws, int slot, size_t n, T** out) {
  auto& b = ws[slot];
  const size_t bytes = (n ? n : 1) * sizeof(T);
  if (b.cap < bytes) {
    (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    HIP_TRY(hipMalloc(&b.p, bytes));
    b.cap = bytes;
  }
  *out = (T*)b.p;
  return 0;
}
template <class T>
static int ws_get(lddl_ctx* c, int slot, size_t n, T** out) {
  return ws_get(c->ws, slot, n, out);
}
static void free_pack(lddl_pack* k) {
  for (auto& b : k->ws) {
    (void)hipFree(b.p);
    b = WsBuf{};
  }
}


extern "C" const char* lddl_last_error(void) { return g_err; }

static void free_ctx(lddl_ctx* c) {
  if (!c) return;
  (void)hipFree(c->d_tdbg);
  (void)hipFree(c->d_pdbg);
  (void)hipFree(c->d_top);
  (void)hipFree(c->d_pages);
  (void)hipFree(c->d_bmp);
  (void)hipFree(c->d_xmap);
  (void)hipFree(c->d_multi);
  (void)hipFree(c->d_slots);
  (void)hipFree(c->d_bloom);
  (void)hipFree(c->d_pool);
  (void)hipFree(c->d_voff);
  (void)hipFree(c->d_rpool);
  (void)hipFree(c->d_rinfo);
  (void)hipFree(c->d_vt);
  (void)hipFree(c->d_vbloom);
  (void)hipFree(c->d_st);
  (void)hipFree(c->d_ovf);
  (void)hipFree(c->d_counter);
  (void)hipFree(c->d_ctab);
  (void)hipFree(c->d_nrec);
  (void)hipFree(c->d_trie);
  (void)hipFree(c->d_lane_ctab);
  (void)hipFree(c->d_lane_stats);
  if (c->tm) {
    for (int k = 0; k < 3; ++k)
      for (int j = 0; j < 2; ++j)
        for (int i = 0; i < 64; ++i) (void)hipEventDestroy(c->tm->ev[k][j][i]);
    delete c->tm;
  }
  for (auto& b : c->ws) (void)hipFree(b.p);
  free_pack(&c->own);
  if (c->h_tot) (void)hipHostFree(c->h_tot);
  delete c;
}

extern "C" void lddl_destroy(lddl_ctx* c) {
  if (c) (void)hipSetDevice(c->device);
  free_ctx(c);
}

template <class T>
static int upload(T** dst, const void* src, size_t bytes) {
  HIP_TRY(hipMalloc((void**)dst, bytes ? bytes : 16));
  if (bytes) HIP_TRY(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
  return 0;
}

static int load_table(lddl_ctx* c, const char* path) {
  UniTables T;
  std::string err;
  int rc = build_uni_tables(path, T, err);
  if (rc) return set_err(rc, "%s", err.c_str());
  c->scan_ok = T.scan_ok;
  c->lane_ok = T.lane_ok;
  if ((rc = upload(&c->d_lane_ctab, T.lane_ctab.data(), T.lane_ctab.size() * 2))) return rc;
  if ((rc = upload(&c->d_top, T.top.data(), T.top.size() * 2))) return rc;
  if ((rc = upload(&c->d_pages, T.pages.data(), T.pages.size() * 4))) return rc;
  if ((rc = upload(&c->d_multi, T.multi.data(), T.multi.size() * 4))) return rc;
  if ((rc = upload(&c->d_bmp, T.bmp.data(), T.bmp.size() * 4))) return rc;
  if ((rc = upload(&c->d_xmap, T.xmap.data(), T.xmap.size() * 4))) return rc;
  return 0;
}

static int load_vocab(lddl_ctx* c, const char* path) {
  VocabTables V;
  std::string err;
  // the trie only for the options that read it (its build is the bulk of
  // the table setup)
  const char* algo = getenv("LDDL_TOKENIZE_ALGO");
  const char* wp = getenv("LDDL_WP_ALGO");
  const bool want_trie = (algo && algo[0] == '6') || (wp && strcmp(wp, "trie") == 0);
  int rc = build_vocab_tables(path, V, err, want_trie);
  if (rc) return set_err(rc, "%s", err.c_str());
  c->vocab_size = (int)V.vocab.size();
  for (int k = 0; k < 5; ++k) c->special[k] = V.special[k];
  c->maxb[0] = V.maxb[0];
  c->maxb[1] = V.maxb[1];
  c->slot_mask = V.slot_mask;
  c->vt_mask = V.vt_mask;
  if ((rc = upload(&c->d_bloom, V.bloom.data(), V.bloom.size() * 4))) return rc;
  if ((rc = upload(&c->d_vt, V.vt.data(), V.vt.size() * 4))) return rc;
  if ((rc = upload(&c->d_vbloom, V.vbloom.data(), V.vbloom.size() * 4))) return rc;
  c->st_mask = V.st_mask;
  if ((rc = upload(&c->d_st, V.st.data(), V.st.size() * 4))) return rc;
  if ((rc = upload(&c->d_slots, V.slots.data(), V.slots.size() * sizeof(uint4)))) return rc;
  if ((rc = upload(&c->d_pool, V.pool.data(), V.pool.size()))) return rc;
  if ((rc = upload(&c->d_voff, V.voff.data(), V.voff.size() * 4))) return rc;
  if ((rc = upload(&c->d_rpool, V.rpool.data(), V.rpool.size()))) return rc;
  if ((rc = upload(&c->d_rinfo, V.rinfo.data(), V.rinfo.size() * 4))) return rc;
  if (V.trie.empty()) {
    c->lane_ok = false;
  } else {
    if ((rc = upload(&c->d_trie, V.trie.data(), V.trie.size() * sizeof(uint2)))) return rc;
    c->trie_base[0] = V.trie_base[0];
    c->trie_base[1] = V.trie_base[1];
  }
  c->vocab = std::move(V.vocab);
  return 0;
}

// the tokenizer algorithm: the one asked for, or the serial path (0) when it
// does not model the loaded tables (the lane tokenizer needs the trie and a
// table in which no code point normalises to more chars than its UTF-8
// bytes; the split one keeps ids below SPLIT_EDEF and derives its byte
// classes from the ASCII page)
static void select_tok_algo(lddl_ctx* c, int algo) {
  c->tok_algo = algo;
  if (c->tok_algo == 6 && !c->lane_ok) c->tok_algo = 0;
  if (c->tok_algo == 5 && (!c->scan_ok || c->vocab_size > (int)SPLIT_EDEF)) c->tok_algo = 0;
}

extern "C" int lddl_create(const char* vocab_path, const char* table_path, int device, lddl_ctx** out) {
  if (!out || !vocab_path || !table_path) return set_err(LDDL_EINVAL, "null argument");
  *out = nullptr;
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return set_err(LDDL_EINVAL, "device %d out of range (%d devices)", device, ndev);
  HIP_TRY(hipSetDevice(device));
  lddl_ctx* c = new lddl_ctx();
  c->device = device;
  int rc = 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) { free_ctx(c); return set_err(LDDL_EHIP, "hipGetDeviceProperties"); }
  c->n_cu = prop.multiProcessorCount;
  if ((rc = load_table(c, table_path)) || (rc = load_vocab(c, vocab_path))) { free_ctx(c); return rc; }
  // 5: the split tokenizer (default); 6: the lane tokenizer of round 5
  // (measured slower; A/B); 0: every tile through the exact serial
  // path -- LDDL_TOKENIZE_ALGO selects (tests); an algorithm that does not model the tables falls back
  // to the serial one (the lane tokenizer needs the trie and a table in which
  // no code point normalises to more chars than its UTF-8 bytes; the split
  // one keeps ids below SPLIT_EDEF and derives its byte classes from the
  // ASCII page)
  const char* algo = getenv("LDDL_TOKENIZE_ALGO");
  select_tok_algo(c, !algo ? 5 : algo[0] == '0' ? 0 : algo[0] == '6' ? 6 : 5);
  const char* mcap = getenv("LDDL_MLM_CAP");  // initial masking arena (tests force the regrow path)
  c->mlm_cap0 = mcap ? (uint64_t)atoll(mcap) : 0;
  c->own.device = device;
  c->own.mlm_cap = c->mlm_cap0;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, tokenize_fallback_kernel_ptr(), 256, 0) != hipSuccess ||
      per_cu < 1)
    per_cu = 4;
  c->tok_grid = c->n_cu * per_cu;
  const size_t ovf_bytes = (size_t)c->tok_grid * 256 * WB_OVF;
  if (hipMalloc((void**)&c->d_ovf, ovf_bytes) != hipSuccess ||
      hipMalloc((void**)&c->d_counter, 64) != hipSuccess) {
    free_ctx(c);
    return set_err(LDDL_ENOMEM, "scratch allocation failed");
  }
  *out = c;
  return 0;
}

extern "C" int lddl_vocab_size(const lddl_ctx* c) { return c ? c->vocab_size : set_err(LDDL_EINVAL, "null ctx"); }

extern "C" int lddl_special_ids(const lddl_ctx* c, int32_t out[5]) {
  if (!c || !out) return set_err(LDDL_EINVAL, "null argument");
  for (int k = 0; k < 5; ++k) out[k] = (int32_t)c->special[k];
  return 0;
}

extern "C" int lddl_vocab_token(const lddl_ctx* c, int32_t id, char* buf, int64_t cap) {
  if (!c || !buf) return set_err(LDDL_EINVAL, "null argument");
  if (id < 0 || id >= c->vocab_size) return set_err(LDDL_EINVAL, "id %d out of range", id);
  const std::string& w = c->vocab[id];
  if ((int64_t)w.size() + 1 > cap) return set_err(LDDL_EINVAL, "buffer too small");
  memcpy(buf, w.data(), w.size());
  buf[w.size()] = 0;
  return (int)w.size();
}

extern "C" int lddl_tokenize(lddl_ctx* c, const uint8_t* d_bytes, int64_t nbytes, const int64_t* d_sent_off,
                             int64_t n_sent, int32_t max_tok, uint16_t* d_out_ids, int64_t out_cap,
                             int32_t* d_out_ntok, int64_t* d_out_tok_off, void* stream) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  if (n_sent < 0 || max_tok < 1 || max_tok > 65534 || nbytes < 0 || out_cap < 0)
    return set_err(LDDL_EINVAL, "n_sent %lld nbytes %lld max_tok %d out_cap %lld", (long long)n_sent,
                   (long long)nbytes, max_tok, (long long)out_cap);
  if (!d_out_tok_off) return set_err(LDDL_EINVAL, "null device pointer");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  if (n_sent == 0) {
    HIP_TRY(hipMemsetAsync(d_out_tok_off, 0, sizeof(int64_t), st));
    return 0;
  }
  if (!d_bytes || !d_sent_off || (!d_out_ids && out_cap > 0) || !d_out_ntok)
    return set_err(LDDL_EINVAL, "null device pointer");
  TokParams P{};
  P.bytes = d_bytes;
  P.sent_off = d_sent_off;
  P.n_sent = n_sent;
  P.max_tok = max_tok;
  P.out_ids = d_out_ids;
  P.out_ntok = d_out_ntok;
  P.out_tok_off = d_out_tok_off;
  P.out_cap = out_cap;
  c->spec_ids = nullptr;
  if (c->spec_flags) {
    int rc;
    if ((rc = ws_get(c, 41, n_sent, &P.sent_spec))) return rc;
    c->spec_ids = d_out_ids;
    c->spec_ntok = d_out_ntok;
    c->spec_soff = d_sent_off;
    c->spec_nsent = n_sent;
  }
  P.top = c->d_top;
  P.pages = c->d_pages;
  P.bmp = c->d_bmp;
  P.xmap = c->d_xmap;
  P.multi = c->d_multi;
  P.slots = c->d_slots;
  P.slot_mask = c->slot_mask;
  P.bloom = c->d_bloom;
  P.pool = c->d_pool;
  P.voff = c->d_voff;
  P.maxb[0] = c->maxb[0];
  P.maxb[1] = c->maxb[1];
  for (int k = 0; k < 5; ++k) P.special[k] = c->special[k];
  P.unk = c->special[1];
  P.vt = c->d_vt;
  P.vt_mask = c->vt_mask;
  P.vbloom = c->d_vbloom;
  // LDDL_SCAN_TABLE=1: the scan probes its two-choice whole-word table
  // (half the scan's fetch, 3 % fewer WordPiece records, but the scan 3.5 %
  // slower: profiles/r5_scan_table.txt); default: slot 0 of the vt bucket
  {
    const char* e = getenv("LDDL_SCAN_TABLE");
    P.st = (e && e[0] == '1') ? c->d_st : nullptr;
    P.st_mask = c->st_mask;
  }
  P.trie = c->d_trie;
  P.trie_base[0] = c->trie_base[0];
  P.trie_base[1] = c->trie_base[1];
  P.ovf = c->d_ovf;
  P.work_counter = c->d_counter;
  HIP_TRY(hipMemsetAsync(c->d_counter, 0, 64, st));
  const char* dbgenv = getenv("LDDL_TOK_DEBUG");

  if (dbgenv && dbgenv[0] == '1') {
    if (!c->d_tdbg) HIP_TRY(hipMalloc((void**)&c->d_tdbg, 32 * 8));
    HIP_TRY(hipMemsetAsync(c->d_tdbg, 0, 32 * 8, st));
    P.dbg = c->d_tdbg;
  }
  const int64_t nt = tile_count(nbytes);
  // LDDL_SPLIT_SEG (tiles per segment) / LDDL_SPLIT_CHUNKS (record chunks):
  // tests force segment seams and record-capacity fallbacks at small sizes.
  // The serial path (tok_algo 0) is one segment of fallback tiles.
  const char* eseg = getenv("LDDL_SPLIT_SEG");
  const char* ech = getenv("LDDL_SPLIT_CHUNKS");
  const int64_t seg_max = c->tok_algo == 0 ? nt : eseg && atoll(eseg) > 0 ? atoll(eseg) : SPLIT_SEG_TILES;
  const int64_t seg = nt < seg_max ? nt : seg_max;
  const bool split = c->tok_algo == 5;
  int64_t n_chunks = !split ? 1 : split_seg_slots(seg, c->n_cu) / SPLIT_CHUNK;
  if (ech && atoll(ech) > 0 && split) n_chunks = atoll(ech);
  const int64_t slots = n_chunks * SPLIT_CHUNK;
  int64_t* tile_sent;
  SplitParams S{};
  int rc;
  // (the entry / staging buffer: u16 per byte of a segment + the last
  // sentence's ids past its end)
  if ((rc = ws_get(c, 19, nt + 1, &tile_sent)) || (rc = ws_get(c, 20, (size_t)fb_list_cap(seg), &S.fb_list)) ||
      (rc = ws_get(c, 21, 16, &S.fb_count)) ||
      (rc = ws_get(c, 34, (size_t)seg * 1024 + (size_t)max_tok + 4096, &S.ent)) ||
      (rc = ws_get(c, 36, (size_t)n_chunks + 16, &S.chunk_fill)) ||
      (rc = ws_get(c, 45, (size_t)scan_blocks(n_sent) + 1, &S.scan_bsum)))
    return rc;
  // (the serial path (0) runs the split path's finish: count / expand read
  // smeta, snslot, cnt8 and, unconditionally, pch[0] -- one chunk of them)
  if (c->tok_algo != 6 &&
      ((rc = ws_get(c, 35, (size_t)slots * 4, &S.rec)) || (rc = ws_get(c, 42, (size_t)slots * 4, &S.pcs)) ||
       (rc = ws_get(c, 47, (size_t)slots, &S.pch)) || (rc = ws_get(c, 37, n_sent, &S.smeta)) ||
       (rc = ws_get(c, 43, n_sent, &S.snslot)) || (rc = ws_get(c, 44, (size_t)slots, &S.cnt8))))
    return rc;
  // (the finish pass -- count_kernel and expand_kernel of algorithms 5 and 0
  // -- reads these unconditionally: refuse to run it without them)
  if (c->tok_algo != 6 && (!S.pch || !S.smeta || !S.snslot || !S.cnt8 || !S.rec || !S.pcs))
    return set_err(LDDL_EINVAL, "tokenize: finish scratch not allocated");
  int64_t* tile_off = nullptr;
  if (c->tok_algo == 6 && (rc = ws_get(c, 46, nt + 1, &tile_off))) return rc;  // (the lane tokenizer's tile starts)
  S.tile_off = tile_off;
  S.chunk_ctr = S.chunk_fill + n_chunks;
  S.n_chunks = (uint32_t)n_chunks;
  S.seg_tiles = seg;
  S.seg_sent_cap = n_sent;
  S.n_fallback = c->d_counter + 8;
  if (c->timing) {
    S.n_rec = c->d_nrec;
    HIP_TRY(hipMemsetAsync(c->d_nrec, 0, 8, st));
  }
  c->last_tok_bytes = nbytes;
  c->last_tok_sent = n_sent;
  if (c->tok_algo == 0) {
    HIP_TRY(launch_tokenize_serial_dense(P, nbytes, tile_sent, S, c->n_cu, c->tok_grid, st));
  } else if (c->tok_algo == 6) {
    tok6::LaneParams Q{};
    Q.trie = c->d_trie;
    Q.rbase[0] = c->trie_base[0];
    Q.rbase[1] = c->trie_base[1];
    if (getenv("LDDL_LANE_STATS")) {
      if (!c->d_lane_stats) HIP_TRY(hipMalloc((void**)&c->d_lane_stats, 64));
      HIP_TRY(hipMemsetAsync(c->d_lane_stats, 0, 64, st));
      Q.stats = c->d_lane_stats;
    }
    HIP_TRY(launch_tokenize_lane(P, nbytes, tile_sent, S, Q, c->d_lane_ctab, c->n_cu, c->tok_grid, st,
                                 c->timing ? c->tm : nullptr));
    if (Q.stats) {
      uint64_t h[7];
      HIP_TRY(hipMemcpyAsync(h, Q.stats, sizeof h, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      fprintf(stderr, "[lddl tok6] lane-iterations %llu busy %.4f slow passes %llu ticks handout %llu refill %llu "
              "slow %llu step %llu\n", (unsigned long long)h[0], h[0] ? (double)h[1] / (double)h[0] : 0.0,
              (unsigned long long)h[2], (unsigned long long)h[3], (unsigned long long)h[4], (unsigned long long)h[5],
              (unsigned long long)h[6]);
    }
  } else {
    HIP_TRY(launch_tokenize_split(P, nbytes, tile_sent, S, c->n_cu, c->tok_grid, st,
                                  c->timing ? c->tm : nullptr));
  }
  if (P.dbg) {
    uint64_t h[24];
    HIP_TRY(hipMemcpyAsync(h, P.dbg, sizeof h, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const char* nm[12] = {"loop", "setup", "classify", "except", "units", "urec", "prep", "probe", "records",
                          "tile_end", "entries", "tiles"};
    fprintf(stderr, "[lddl tok5 dbg] ntiles=%lld", (long long)nt);
    for (int k = 0; k < 12; ++k) fprintf(stderr, " %s=%llu", nm[k], (unsigned long long)h[k]);
    const char* wn[6] = {"wp_A", "wp_B", "wp_C", "wp_D", "wp_steps", "wp_lane_steps"};
    for (int k = 0; k < 6; ++k) fprintf(stderr, " %s=%llu", wn[k], (unsigned long long)h[12 + k]);
    fprintf(stderr, " prep_decode=%llu prep_dirty=%llu x_list=%llu x_load=%llu x_apply=%llu", (unsigned long long)h[18],
            (unsigned long long)h[19], (unsigned long long)h[20], (unsigned long long)h[21], (unsigned long long)h[22]);
    fprintf(stderr, "\n");
  }
  return 0;
}

extern "C" int lddl_set_special_flags(lddl_ctx* c, int on) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  c->spec_flags = on != 0;
  return 0;
}

extern "C" int lddl_set_tokenize_algo(lddl_ctx* c, int algo, int* out_algo) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  if (algo != 0 && algo != 5 && algo != 6) return set_err(LDDL_EINVAL, "tokenize algo must be 0, 5 or 6");
  select_tok_algo(c, algo);
  if (out_algo) *out_algo = c->tok_algo;
  return 0;
}

extern "C" int lddl_set_timing(lddl_ctx* c, int on) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  HIP_TRY(hipSetDevice(c->device));
  if (on && !c->tm) {
    c->tm = new SplitTiming();
    for (int k = 0; k < 3; ++k)
      for (int j = 0; j < 2; ++j)
        for (int i = 0; i < 64; ++i) HIP_TRY(hipEventCreate(&c->tm->ev[k][j][i]));
    HIP_TRY(hipMalloc((void**)&c->d_nrec, 16));
  }
  c->timing = on != 0;
  return 0;
}

extern "C" int lddl_tokenize_stats(lddl_ctx* c, double* out, int n) {
  if (!c || !out || n < 6) return set_err(LDDL_EINVAL, "need out[6]");
  if (!c->timing || !c->tm) return set_err(LDDL_EINVAL, "timing is off (lddl_set_timing)");
  HIP_TRY(hipSetDevice(c->device));
  for (int k = 0; k < 3; ++k) {
    double ms = 0.0;
    for (int i = 0; i < c->tm->n[k]; ++i) {
      HIP_TRY(hipEventSynchronize(c->tm->ev[k][1][i]));
      float f = 0.0f;
      HIP_TRY(hipEventElapsedTime(&f, c->tm->ev[k][0][i], c->tm->ev[k][1][i]));
      ms += f;
    }
    out[k] = ms;
  }
  unsigned long long nrec = 0;
  HIP_TRY(hipMemcpy(&nrec, c->d_nrec, 8, hipMemcpyDeviceToHost));
  out[3] = (double)nrec;
  out[4] = (double)c->tm->n[0];
  uint32_t nfb = 0;
  HIP_TRY(hipMemcpy(&nfb, c->d_counter + 8, 4, hipMemcpyDeviceToHost));
  out[5] = (double)nfb;
  return 0;
}

static int pack_common(lddl_ctx* c, lddl_pack* pk, int codebert, const int32_t* d_ntok, const int64_t* d_tok_off,
                       const int64_t* d_sent_off, int64_t n_sent,
                       const int64_t* d_doc_sent_off, const int32_t* d_doc_nseg_doc, int64_t n_doc,
                       const int64_t* d_part_doc_off, int64_t n_part, int32_t target_seq_length,
                       double short_seq_prob, int32_t duplicate_factor, uint64_t seed, int32_t bin_size,
                       int64_t* out_totals, void* stream, const uint16_t* d_ids = nullptr, int32_t masking = 0,
                       double masked_lm_ratio = 0.15) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  lddl_pack* k = pk ? pk : &c->own;
  if (k->device != c->device) return set_err(LDDL_EINVAL, "pack result of another device");
  if (masking) {
    if (!d_ids) return set_err(LDDL_EINVAL, "masking needs the tokenizer ids");
    if (target_seq_length > MLM_MAX_SEQ)
      return set_err(LDDL_EINVAL, "masking supports target_seq_length <= %d", MLM_MAX_SEQ);
    if (!(masked_lm_ratio >= 0.0 && masked_lm_ratio <= 1.0))
      return set_err(LDDL_EINVAL, "masked_lm_ratio %g not in [0, 1]", masked_lm_ratio);
    if (c->vocab_size > 65535) return set_err(LDDL_EINVAL, "masking: vocab larger than 65535");
  }
  if (n_part < 1 || n_doc < 0 || n_sent < 0) return set_err(LDDL_EINVAL, "bad sizes");
  if (!d_ntok || !d_tok_off || !d_sent_off || !d_doc_sent_off || !d_part_doc_off || !out_totals)
    return set_err(LDDL_EINVAL, "null pointer");
  if (codebert && !d_doc_nseg_doc) return set_err(LDDL_EINVAL, "codebert needs doc_nseg_doc");
  if (target_seq_length < 5 || target_seq_length > 32768)
    return set_err(LDDL_EINVAL, "target_seq_length %d not in [5, 32768]", target_seq_length);
  if (duplicate_factor < 1) return set_err(LDDL_EINVAL, "duplicate_factor %d < 1", duplicate_factor);
  int32_t nbins = 1;
  if (bin_size > 0) {
    // pretrain.py:566-571
    if (bin_size > target_seq_length) return set_err(LDDL_EINVAL, "bin size must be <= target-seq-length");
    if (target_seq_length % bin_size) return set_err(LDDL_EINVAL, "bin size must divide target-seq-length");
    nbins = target_seq_length / bin_size;
  } else {
    bin_size = 1 << 30;
  }
  if (nbins > 255) return set_err(LDDL_EINVAL, "more than 255 bins");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  k->last_npairs = -1;  // until this pack succeeds, nothing to materialise
  k->last_nmask = -1;
  k->last_tokens = nullptr;
  PackParams& P = k->pp;
  P = PackParams{};
  P.ntok = d_ntok;
  P.sent_off = d_sent_off;
  P.doc_sent_off = d_doc_sent_off;
  P.part_doc_off = d_part_doc_off;
  P.doc_nseg_doc = d_doc_nseg_doc;
  P.n_part = n_part;
  P.max_seq = target_seq_length;
  P.dup = duplicate_factor;
  P.short_seq_prob = short_seq_prob;
  P.seed = seed;
  P.bin_size = bin_size;
  P.nbins = nbins;
  const size_t npair_cap = (size_t)duplicate_factor * (size_t)(n_sent ? n_sent : 1);
  int rc;
  if ((rc = ws_get(k->ws, 0, n_sent, &P.fs_ntok)) || (rc = ws_get(k->ws, 1, n_sent, &P.fs_base)) ||
      (rc = ws_get(k->ws, 2, n_doc, &P.fd_first)) || (rc = ws_get(k->ws, 3, n_doc, &P.fd_n)) ||
      (rc = ws_get(k->ws, 4, n_doc, &P.fd_nd)) ||
      (rc = ws_get(k->ws, 6, npair_cap, &P.pairs)) || (rc = ws_get(k->ws, 7, npair_cap, &P.order)) ||
      (rc = ws_get(k->ws, 8, npair_cap, &P.binned)) || (rc = ws_get(k->ws, 9, npair_cap, &P.tok_local)) ||
      (rc = ws_get(k->ws, 10, n_part, &P.part_npairs)) || (rc = ws_get(k->ws, 11, n_part, &P.part_ntok)) ||
      (rc = ws_get(k->ws, 12, (size_t)n_part * nbins, &P.bin_count)) ||
      (rc = ws_get(k->ws, 13, (size_t)n_part * nbins, &P.bin_cursor)) ||
      (rc = ws_get(k->ws, 14, n_part, &P.part_err)) || (rc = ws_get(k->ws, 18, n_sent + n_part + 1, &P.kept)) ||
      (rc = ws_get(k->ws, 33, n_sent, &P.fs_dense)))
    return rc;
  {
    uint32_t* mts;
    if ((rc = ws_get(k->ws, 19, (size_t)((n_part + 63) & ~(int64_t)63) * MT_N, &mts))) return rc;  // (whole 64-partition rows)
    HIP_TRY(launch_mt_seed_states(seed, n_part, mts, st));
    P.mt_states = mts;
  }
  P.tokoff = d_tok_off;  // the tokenizer's dense offsets (lddl_tokenize d_out_tok_off)
  int64_t *pair_base, *tok_base;
  int32_t* err_any;
  if ((rc = ws_get(k->ws, 15, n_part + 1, &pair_base)) || (rc = ws_get(k->ws, 16, n_part + 1, &tok_base)) ||
      (rc = ws_get(k->ws, 17, 4, &err_any)))
    return rc;
  if (!c->h_tot) HIP_TRY(hipHostMalloc((void**)&c->h_tot, 8 * sizeof(int64_t)));
  int64_t *mask_base = nullptr, *mask_base2 = nullptr;
  if (masking) {
    P.masking = 1;
    P.mlm_ratio = masked_lm_ratio;
    P.n_vocab = (uint32_t)c->vocab_size;
    P.cls_id = c->special[2];
    P.sep_id = c->special[3];
    P.mask_id = c->special[4];
    P.ids = d_ids;
    uint8_t *sent_spec, *fs_spec;
    // the flags of the last lddl_tokenize into these buffers, else a pass over the ids
    // (one pack consumes them: a later pack over recycled buffers at the same
    // addresses recomputes the flags from the ids)
    const bool spec_ok = c->spec_ids == d_ids && c->spec_ntok == d_ntok && c->spec_soff == d_sent_off &&
                         c->spec_nsent == n_sent;
    c->spec_ids = nullptr;
    if ((rc = spec_ok ? ws_get(c->ws, 41, n_sent, &sent_spec) : ws_get(k->ws, 22, n_sent, &sent_spec)) ||
        (rc = ws_get(k->ws, 23, n_sent, &fs_spec)) ||
        (rc = ws_get(k->ws, 24, npair_cap, &P.mref)) || (rc = ws_get(k->ws, 25, npair_cap, &P.mloc)) ||
        (rc = ws_get(k->ws, 26, n_part, &P.part_nmask)) || (rc = ws_get(k->ws, 27, n_part + 1, &mask_base)) ||
        (rc = ws_get(k->ws, 28, n_part + 1, &mask_base2)) || (rc = ws_get(k->ws, 29, 1, &P.mcounter)) ||
        (rc = ws_get(k->ws, 31, (size_t)n_part * MLM_MAX_SEQ, &P.mcand)))
      return rc;
    P.sent_spec = sent_spec;
    P.fs_spec = fs_spec;
    if (!spec_ok) HIP_TRY(launch_sent_special(d_ids, d_tok_off, d_ntok, n_sent, P.cls_id, P.sep_id, sent_spec, st));
    if (!k->mlm_cap) k->mlm_cap = (uint64_t)n_part * 4 * MLM_CHUNK + (uint64_t)duplicate_factor * n_sent * 4;
  }
  if (!codebert) {
    // Wave packer: one 64-lane workgroup per partition runs a serial chain, so
    // throughput is partitions in flight; measured on the bench workload the
    // per-partition arrays are best left in global memory (L2), keeping the
    // workgroup at ~5 KiB of LDS (~30 partitions per CU): 65 ms against 250 ms
    // with 4 partitions per CU.  LDDL_PACK_CAPS=lens,docs,pairs puts them in LDS.
    P.cap_lens = 0;
    P.cap_docs = 0;
    P.cap_pairs = 0;
    const char* caps = getenv("LDDL_PACK_CAPS");  // "lens,docs,pairs" override (tuning)
    if (caps) {
      int a = 0, b = 0, d = 0;
      if (sscanf(caps, "%d,%d,%d", &a, &b, &d) == 3) {
        P.cap_lens = a / 64 * 64;
        P.cap_docs = b / 64 * 64;
        P.cap_pairs = std::min(d / 64 * 64, 65472);
      }
    }
  }
  for (int attempt = 0;; ++attempt) {
    if (masking) {
      if ((rc = ws_get(k->ws, 30, k->mlm_cap, &P.marena))) return rc;
      P.mcap = k->mlm_cap;
      HIP_TRY(hipMemsetAsync(P.mcounter, 0, 8, st));
    }
    const char* pdbg = getenv("LDDL_PACK_DEBUG");
    P.dbg = nullptr;
    const int64_t pdbg_n = 16 + 2 * (int64_t)n_part;  // counters + the BERT packer's per-wave start / end
    if (pdbg && pdbg[0] == '1') {
      if (c->pdbg_cap < pdbg_n) {
        (void)hipFree(c->d_pdbg);
        c->d_pdbg = nullptr;
        c->pdbg_cap = 0;
        HIP_TRY(hipMalloc((void**)&c->d_pdbg, pdbg_n * 8));
        c->pdbg_cap = pdbg_n;
      }
      HIP_TRY(hipMemsetAsync(c->d_pdbg, 0, pdbg_n * 8, st));
      P.dbg = c->d_pdbg;
    }
    HIP_TRY(codebert ? launch_pack_codebert_wave(P, st) : launch_pack_bert_wave(P, st));
    if (P.dbg && !codebert) {
      uint64_t h[16];
      HIP_TRY(hipMemcpyAsync(h, P.dbg, sizeof h, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      const char* nm[16] = {"filter", "ldsfill", "seed", "generate", "shuffle", "bin", "pairs", "parts",
                            "m_cand", "m_draws", "m_trace", "m_choices", "m_write", "m_trace_fbuild", "m_trace_chains",
                            "unused"};
      const char* gn[5] = {"g_doc", "g_fill", "g_pairB", "g_trunc", "g_store"};  // unmasked: generate sub-phases
      fprintf(stderr, "[lddl pack dbg]");
      for (int k = 0; k < (P.masking ? 15 : 13); ++k)
        fprintf(stderr, " %s=%llu", k < 8 || P.masking ? nm[k] : gn[k - 8], (unsigned long long)h[k]);
      fprintf(stderr, "\n");
      // occupancy timeline (100 MHz ticks): the span from the first wave's
      // start to the last one's end, the summed wave time, the most waves
      // resident at once, and how long the residency stays below 90 % / 50 %
      // of that maximum after the peak (the tail)
      std::vector<uint64_t> tl(2 * (size_t)n_part);
      HIP_TRY(hipMemcpyAsync(tl.data(), P.dbg + 16, tl.size() * 8, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      std::vector<std::pair<uint64_t, int>> ev;
      ev.reserve(tl.size());
      uint64_t busy = 0, t_lo = ~0ull, t_hi = 0;
      for (int64_t q = 0; q < n_part; ++q) {
        const uint64_t a = tl[2 * q], b = tl[2 * q + 1];
        if (b < a || a == 0) continue;
        ev.push_back({a, 1});
        ev.push_back({b, -1});
        busy += b - a;
        t_lo = std::min(t_lo, a);
        t_hi = std::max(t_hi, b);
      }
      std::sort(ev.begin(), ev.end());
      int cur = 0, mx = 0;
      uint64_t t_peak = t_lo;
      for (auto& e : ev) {
        cur += e.second;
        if (cur > mx) { mx = cur; t_peak = e.first; }
      }
      uint64_t below90 = 0, below50 = 0, prev = t_lo;
      cur = 0;
      for (auto& e : ev) {
        if (e.first > t_peak) {
          if (cur < 0.9 * mx) below90 += e.first - prev;
          if (cur < 0.5 * mx) below50 += e.first - prev;
        }
        prev = e.first;
        cur += e.second;
      }
      std::vector<uint64_t> du;
      uint64_t last_start = 0;
      for (int64_t q = 0; q < n_part; ++q)
        if (tl[2 * q] && tl[2 * q + 1] >= tl[2 * q]) {
          du.push_back(tl[2 * q + 1] - tl[2 * q]);
          last_start = std::max(last_start, tl[2 * q] - t_lo);
        }
      std::sort(du.begin(), du.end());
      auto pct = [&](double f) { return du.empty() ? 0.0 : du[std::min(du.size() - 1, (size_t)(f * du.size()))] / 100.0; };
      fprintf(stderr, "[lddl pack tl] wave_us p10=%.0f p50=%.0f p90=%.0f max=%.0f last_start_us=%.0f\n", pct(0.1), pct(0.5),
              pct(0.9), pct(1.0), last_start / 100.0);
      fprintf(stderr, "[lddl pack tl] waves=%zu span_us=%.0f busy_wave_us=%.0f max_resident=%d mean_resident=%.0f tail_below90_us=%.0f tail_below50_us=%.0f mean_wave_us=%.0f\n",
              ev.size() / 2, (t_hi - t_lo) / 100.0, busy / 100.0, mx, t_hi > t_lo ? (double)busy / (double)(t_hi - t_lo) : 0.0,
              below90 / 100.0, below50 / 100.0, ev.empty() ? 0.0 : busy / 100.0 / (ev.size() / 2));
    }
    HIP_TRY(launch_scan_parts(P.part_npairs, P.part_ntok, n_part, pair_base, tok_base, P.part_err, err_any, st));
    HIP_TRY(hipMemcpyAsync(c->h_tot, pair_base + n_part, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(c->h_tot + 1, tok_base + n_part, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(c->h_tot + 2, err_any, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(c->h_tot + 5, P.tokoff + n_sent, 8, hipMemcpyDeviceToHost, st));
    if (masking) {
      HIP_TRY(launch_scan_parts(P.part_nmask, P.part_nmask, n_part, mask_base, mask_base2, P.part_err, err_any, st));
      HIP_TRY(hipMemcpyAsync(c->h_tot + 3, mask_base + n_part, 8, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipMemcpyAsync(c->h_tot + 4, P.mcounter, 8, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    // the bump allocator overshot the arena: grow it and pack again (the
    // pack is deterministic, so the rerun reproduces the same rows)
    if (masking && (uint64_t)c->h_tot[4] > k->mlm_cap && attempt == 0) {
      k->mlm_cap = (uint64_t)c->h_tot[4] + (uint64_t)n_part * MLM_CHUNK;
      continue;
    }
    if (masking && (uint64_t)c->h_tot[4] > k->mlm_cap) return set_err(LDDL_ECAPACITY, "masking arena overflow");
    break;
  }
  const int32_t e = (int32_t)(c->h_tot[2] & 0xFFFFFFFF);
  k->pack_codebert = codebert;
  k->last_nmask = masking ? c->h_tot[3] : -1;
  if (e & PACK_EINDEX) { k->last_npairs = -1; return set_err(LDDL_EINDEX, "IndexError in _truncate_seq (reference quirk)"); }
  if (e & PACK_EASSERT) { k->last_npairs = -1; return set_err(LDDL_EASSERT, "AssertionError: empty segment after truncation"); }
  k->last_npairs = c->h_tot[0];
  k->last_ntok = c->h_tot[1];
  k->last_nsent = n_sent;
  k->last_ndense = c->h_tot[5];
  out_totals[0] = k->last_npairs;
  out_totals[1] = k->last_ntok;
  out_totals[2] = nbins;
  out_totals[3] = masking ? k->last_nmask : 0;
  return 0;
}

extern "C" int lddl_pack_bert(lddl_ctx* c, lddl_pack* pk, const uint16_t* d_ids, const int32_t* d_ntok, const int64_t* d_tok_off,
                              const int64_t* d_sent_off, int64_t n_sent, const int64_t* d_doc_sent_off, int64_t n_doc,
                              const int64_t* d_part_doc_off, int64_t n_part, int32_t target_seq_length,
                              double short_seq_prob, int32_t duplicate_factor, int32_t masking,
                              double masked_lm_ratio, uint64_t seed, int32_t bin_size, int64_t* out_totals,
                              void* stream) {
  return pack_common(c, pk, 0, d_ntok, d_tok_off, d_sent_off, n_sent, d_doc_sent_off, nullptr, n_doc, d_part_doc_off, n_part,
                     target_seq_length, short_seq_prob, duplicate_factor, seed, bin_size, out_totals, stream, d_ids,
                     masking, masked_lm_ratio);
}

extern "C" int lddl_pack_codebert(lddl_ctx* c, lddl_pack* pk, const int32_t* d_ntok, const int64_t* d_tok_off,
                                  const int64_t* d_sent_off, int64_t n_sent,
                                  const int64_t* d_doc_sent_off, const int32_t* d_doc_nseg_doc, int64_t n_doc,
                                  const int64_t* d_part_doc_off, int64_t n_part, int32_t target_seq_length,
                                  double short_seq_prob, int32_t duplicate_factor, uint64_t seed, int32_t bin_size,
                                  int64_t* out_totals, void* stream) {
  return pack_common(c, pk, 1, d_ntok, d_tok_off, d_sent_off, n_sent, d_doc_sent_off, d_doc_nseg_doc, n_doc, d_part_doc_off,
                     n_part, target_seq_length, short_seq_prob, duplicate_factor, seed, bin_size, out_totals, stream);
}

// MatParams of the last pack call (lddl_materialize / lddl_row_spans)
static MatParams mat_params(const lddl_ctx* c, const lddl_pack* k) {
  const PackParams& P = k->pp;
  MatParams M{};
  M.fs_dense = P.fs_dense;
  M.sent_off = P.sent_off;
  M.doc_sent_off = P.doc_sent_off;
  M.part_doc_off = P.part_doc_off;
  M.fs_base = P.fs_base;
  M.fs_ntok = P.fs_ntok;
  M.pairs = P.pairs;
  M.binned = P.binned;
  M.tok_local = P.tok_local;
  M.part_npairs = P.part_npairs;
  M.pair_base = (const int64_t*)k->ws[15].p;
  M.tok_base = (const int64_t*)k->ws[16].p;
  M.n_part = P.n_part;
  M.dup = P.dup;
  M.bin_size = P.bin_size;
  M.nbins = P.nbins;
  M.cls_id = c->special[2];
  M.sep_id = c->special[3];
  M.codebert = k->pack_codebert;
  return M;
}

extern "C" int lddl_materialize(lddl_ctx* c, lddl_pack* pk, const uint16_t* d_ids, uint16_t* d_out_tokens, int64_t* d_out_tok_off,
                                uint16_t* d_out_len0, uint16_t* d_out_len1, uint8_t* d_out_flags, uint8_t* d_out_bin,
                                int64_t* d_out_part, int64_t* d_bin_count, void* stream) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  lddl_pack* k = pk ? pk : &c->own;
  if (k->device != c->device) return set_err(LDDL_EINVAL, "pack result of another device");
  if (k->last_npairs < 0) return set_err(LDDL_EINVAL, "no successful lddl_pack_* call to materialise");
  if (!d_ids || !d_out_tokens || !d_out_tok_off || !d_out_len0 || !d_out_len1 || !d_out_flags || !d_out_bin ||
      !d_out_part)
    return set_err(LDDL_EINVAL, "null pointer");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  const PackParams& P = k->pp;
  // LDDL_MAT_ALGO=1: the wave-per-partition materialize kernel (also taken
  // for unaligned buffers); otherwise the chunked v2 kernel
  const int mat_algo = getenv("LDDL_MAT_ALGO") ? atoi(getenv("LDDL_MAT_ALGO")) : 2;
  MatParams M = mat_params(c, k);
  M.dense = d_ids;
  M.out_tokens = d_out_tokens;
  M.out_tok_off = d_out_tok_off;
  M.out_len0 = d_out_len0;
  M.out_len1 = d_out_len1;
  M.out_flags = d_out_flags;
  M.out_bin = d_out_bin;
  M.out_part = d_out_part;
  if (k->last_npairs == 0) {
    HIP_TRY(hipMemsetAsync(d_out_tok_off, 0, 8, st));
  } else {
    HIP_TRY(launch_materialize(M, k->last_npairs, k->last_ndense + 16, mat_algo, st));
  }
  if (d_bin_count)
    HIP_TRY(hipMemcpyAsync(d_bin_count, P.bin_count, (size_t)P.n_part * P.nbins * 8, hipMemcpyDeviceToDevice, st));
  k->last_tokens = d_out_tokens;
  k->last_tok_off = d_out_tok_off;
  k->last_part = d_out_part;
  return 0;
}

extern "C" int lddl_row_spans(lddl_ctx* c, lddl_pack* pk, int64_t* d_out_src0, int64_t* d_out_src1, int64_t* d_out_tok_off,
                              uint16_t* d_out_len0, uint16_t* d_out_len1, uint8_t* d_out_flags, uint8_t* d_out_bin,
                              int64_t* d_out_part, int64_t* d_bin_count, void* stream) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  lddl_pack* k = pk ? pk : &c->own;
  if (k->device != c->device) return set_err(LDDL_EINVAL, "pack result of another device");
  if (k->last_npairs < 0) return set_err(LDDL_EINVAL, "no successful lddl_pack_* call");
  if (!d_out_src0 || !d_out_src1 || !d_out_len0 || !d_out_len1 || !d_out_flags || !d_out_bin || !d_out_part)
    return set_err(LDDL_EINVAL, "null pointer");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  const PackParams& P = k->pp;
  MatParams M = mat_params(c, k);
  M.out_src0 = d_out_src0;
  M.out_src1 = d_out_src1;
  M.out_tok_off = d_out_tok_off;
  M.out_len0 = d_out_len0;
  M.out_len1 = d_out_len1;
  M.out_flags = d_out_flags;
  M.out_bin = d_out_bin;
  M.out_part = d_out_part;
  if (k->last_npairs == 0) {
    if (d_out_tok_off) HIP_TRY(hipMemsetAsync(d_out_tok_off, 0, 8, st));
  } else {
    int32_t* chunk_part = nullptr;
    int64_t* part_pb = nullptr;
    int rc;
    if ((rc = ws_get(c, 48, (size_t)((k->last_npairs + 63) >> 6), &chunk_part)) ||
        (rc = ws_get(c, 49, (size_t)P.n_part, &part_pb)))
      return rc;
    HIP_TRY(launch_chunk_parts(M.pair_base, P.doc_sent_off, P.part_doc_off, P.dup, P.n_part, chunk_part, part_pb, st));
    M.chunk_part = chunk_part;
    M.part_pb = part_pb;
    HIP_TRY(launch_row_spans(M, k->last_npairs, st));
  }
  if (d_bin_count)
    HIP_TRY(hipMemcpyAsync(d_bin_count, P.bin_count, (size_t)P.n_part * P.nbins * 8, hipMemcpyDeviceToDevice, st));
  return 0;
}

extern "C" int lddl_masked_lm(lddl_ctx* c, lddl_pack* pk, int64_t* d_out_mlm_off, uint16_t* d_out_mlm_pos, uint16_t* d_out_mlm_label,
                              void* stream) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  lddl_pack* k = pk ? pk : &c->own;
  if (k->device != c->device) return set_err(LDDL_EINVAL, "pack result of another device");
  if (k->last_npairs < 0 || k->last_nmask < 0 || !k->last_tokens)
    return set_err(LDDL_EINVAL, "lddl_masked_lm needs lddl_pack_bert(masking=1) then lddl_materialize");
  if (!d_out_mlm_off || (k->last_nmask > 0 && (!d_out_mlm_pos || !d_out_mlm_label)))
    return set_err(LDDL_EINVAL, "null pointer");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  const PackParams& P = k->pp;
  if (k->last_npairs == 0) {
    HIP_TRY(hipMemsetAsync(d_out_mlm_off, 0, 8, st));
  } else {
    MlmParams M{};
    M.doc_sent_off = P.doc_sent_off;
    M.part_doc_off = P.part_doc_off;
    M.pair_base = (const int64_t*)k->ws[15].p;
    M.binned = P.binned;
    M.mref = P.mref;
    M.mloc = P.mloc;
    M.mask_base = (const int64_t*)k->ws[27].p;
    M.marena = P.marena;
    M.n_part = P.n_part;
    M.dup = P.dup;
    M.tokens = k->last_tokens;
    M.tok_off = k->last_tok_off;
    M.row_part = k->last_part;
    M.out_off = d_out_mlm_off;
    M.out_pos = d_out_mlm_pos;
    M.out_label = d_out_mlm_label;
    HIP_TRY(launch_masked_lm(M, k->last_npairs, st));
  }
  k->last_nmask = -1;  // the rows are masked in place exactly once
  return 0;
}

extern "C" int lddl_masked_lm_spans(lddl_ctx* c, lddl_pack* pk, const uint16_t* d_ids, const int64_t* d_src0,
                                    const int64_t* d_src1, const uint16_t* d_len0, const int64_t* d_part,
                                    int64_t* d_out_mlm_off, uint16_t* d_out_mlm_pos, uint16_t* d_out_mlm_label,
                                    uint16_t* d_out_mlm_token, void* stream) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  lddl_pack* k = pk ? pk : &c->own;
  if (k->device != c->device) return set_err(LDDL_EINVAL, "pack result of another device");
  if (k->last_npairs < 0 || k->last_nmask < 0)
    return set_err(LDDL_EINVAL, "lddl_masked_lm_spans needs lddl_pack_bert(masking=1) then lddl_row_spans");
  if (!d_out_mlm_off || (k->last_npairs > 0 && (!d_ids || !d_src0 || !d_src1 || !d_len0 || !d_part)) ||
      (k->last_nmask > 0 && (!d_out_mlm_pos || !d_out_mlm_label || !d_out_mlm_token)))
    return set_err(LDDL_EINVAL, "null pointer");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  const PackParams& P = k->pp;
  if (k->last_npairs == 0) {
    HIP_TRY(hipMemsetAsync(d_out_mlm_off, 0, 8, st));
  } else {
    MlmParams M{};
    M.doc_sent_off = P.doc_sent_off;
    M.part_doc_off = P.part_doc_off;
    M.pair_base = (const int64_t*)k->ws[15].p;
    M.binned = P.binned;
    M.mref = P.mref;
    M.mloc = P.mloc;
    M.mask_base = (const int64_t*)k->ws[27].p;
    M.marena = P.marena;
    M.n_part = P.n_part;
    M.dup = P.dup;
    M.row_part = d_part;
    M.ids = d_ids;
    M.src0 = d_src0;
    M.src1 = d_src1;
    M.len0 = d_len0;
    M.out_off = d_out_mlm_off;
    M.out_pos = d_out_mlm_pos;
    M.out_label = d_out_mlm_label;
    M.out_token = d_out_mlm_token;
    HIP_TRY(launch_masked_lm(M, k->last_npairs, st));
  }
  return 0;
}

extern "C" int lddl_pack_new(lddl_ctx* c, lddl_pack** out) {
  if (!c || !out) return set_err(LDDL_EINVAL, "null pointer");
  lddl_pack* k = new (std::nothrow) lddl_pack;
  if (!k) return set_err(LDDL_ENOMEM, "out of host memory");
  k->device = c->device;
  k->mlm_cap = c->mlm_cap0;
  *out = k;
  return 0;
}

extern "C" void lddl_pack_free(lddl_pack* k) {
  if (!k) return;
  (void)hipSetDevice(k->device);
  free_pack(k);
  delete k;
}

extern "C" int lddl_pack_rows(const lddl_pack* k, int64_t* out_npairs) {
  if (!k || !out_npairs) return set_err(LDDL_EINVAL, "null pointer");
  *out_npairs = k->last_npairs;
  return 0;
}

// ---------------------------------------------------------------- bin ----
extern "C" int lddl_bin(lddl_ctx* c, const int64_t* d_num_tokens, int64_t n, int32_t bin_size, int32_t nbins,
                        int64_t* d_out_perm, int64_t* d_out_bin_counts, void* stream) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  if (n < 0) return set_err(LDDL_EINVAL, "negative row count");
  if (bin_size < 1) return set_err(LDDL_EINVAL, "bin_size %d < 1", bin_size);
  if (nbins < 1 || nbins > 1024) return set_err(LDDL_EINVAL, "nbins %d not in [1, 1024]", nbins);
  if (!d_out_bin_counts || (n > 0 && (!d_num_tokens || !d_out_perm))) return set_err(LDDL_EINVAL, "null pointer");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  const int64_t nh = bin_chunks(n) * nbins;
  int32_t *hist, *err;
  int64_t *base, *bsum;
  int rc;
  if ((rc = ws_get(c, 0, (size_t)(nh ? nh : 1), &hist)) || (rc = ws_get(c, 1, (size_t)nh + 1, &base)) ||
      (rc = ws_get(c, 2, (size_t)scan_blocks(nh) + 1, &bsum)) || (rc = ws_get(c, 3, 1, &err)))
    return rc;
  if (!c->h_tot) HIP_TRY(hipHostMalloc((void**)&c->h_tot, 8 * sizeof(int64_t)));
  HIP_TRY(launch_bin(d_num_tokens, n, bin_size, nbins, hist, base, bsum, d_out_perm, d_out_bin_counts, err, st));
  HIP_TRY(hipMemcpyAsync(&c->h_tot[7], err, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if ((int32_t)(c->h_tot[7] & 0xFFFFFFFF))
    return set_err(LDDL_EINDEX, "IndexError: list index out of range (a length bins below -nbins, binning.py:70-73)");
  return 0;
}

// --------------------------------------------------------------- render --
extern "C" int lddl_render_strings(lddl_ctx* c, const uint16_t* d_tokens, const int64_t* d_row_off,
                                   const uint16_t* d_len0, const uint16_t* d_len1, const uint8_t* d_flags,
                                   int64_t row0, int64_t n_rows, int32_t segment, int32_t codebert,
                                   int64_t* d_out_off, uint8_t* d_out_bytes, int64_t out_cap, int64_t* out_nbytes,
                                   void* stream) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  if (segment < RENDER_SEG0 || segment > RENDER_SPAN) return set_err(LDDL_EINVAL, "segment %d not in 0..3", segment);
  if (row0 < 0 || n_rows < 0) return set_err(LDDL_EINVAL, "negative row range");
  if (!d_tokens || !d_row_off || !d_out_off || !out_nbytes) return set_err(LDDL_EINVAL, "null pointer");
  if (segment != RENDER_ROW && (!d_len0 || (segment == RENDER_SEG1 && (!d_len1 || (codebert && !d_flags)))))
    return set_err(LDDL_EINVAL, "segment %d needs len0/len1%s", segment, codebert ? "/flags" : "");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  RenderParams R{};
  R.tokens = d_tokens;
  R.row_off = d_row_off;
  R.len0 = d_len0;
  R.len1 = d_len1;
  R.flags = d_flags;
  R.row0 = row0;
  R.n_rows = n_rows;
  R.segment = segment;
  R.codebert = codebert;
  R.vinfo = c->d_rinfo;
  R.vpool = c->d_rpool;
  int64_t* bsum;
  int rc;
  if ((rc = ws_get(c, 35, (size_t)n_rows, &R.lens))) return rc;
  if ((rc = ws_get(c, 36, (size_t)scan_blocks(n_rows) + 1, &bsum))) return rc;
  HIP_TRY(launch_render_len(R, c->n_cu, st));
  HIP_TRY(launch_scan_ntok(R.lens, n_rows, d_out_off, bsum, st));
  HIP_TRY(hipMemcpyAsync(&c->h_tot[6], d_out_off + n_rows, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  *out_nbytes = c->h_tot[6];
  if (!d_out_bytes) return 0;  // size query
  if (out_cap < c->h_tot[6])
    return set_err(LDDL_ECAPACITY, "render needs %lld bytes, out_cap %lld", (long long)c->h_tot[6], (long long)out_cap);
  R.out_off = d_out_off;
  R.out = d_out_bytes;
  HIP_TRY(launch_render_bytes(R, c->n_cu, st));
  return 0;
}

extern "C" int lddl_render_npy(lddl_ctx* c, const int64_t* d_mlm_off, const uint16_t* d_mlm_pos, int64_t row0,
                               int64_t n_rows, const uint16_t* d_hdr, int32_t hdr_len, int32_t kmax, int64_t* d_out_off,
                               uint8_t* d_out_bytes, int64_t out_cap, int64_t* out_nbytes, void* stream) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  if (row0 < 0 || n_rows < 0) return set_err(LDDL_EINVAL, "negative row range");
  if (hdr_len <= 0 || (hdr_len & 1) || kmax < 0) return set_err(LDDL_EINVAL, "header length %d must be even and > 0", hdr_len);
  if (!d_out_off || !out_nbytes || (n_rows > 0 && (!d_mlm_off || !d_hdr))) return set_err(LDDL_EINVAL, "null pointer");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  NpyParams N{};
  N.moff = d_mlm_off;
  N.mpos = d_mlm_pos;
  N.row0 = row0;
  N.n_rows = n_rows;
  N.hdr = d_hdr;
  N.hdr_u16 = hdr_len / 2;
  N.kmax = kmax;
  int64_t* bsum;
  int rc;
  if ((rc = ws_get(c, 35, (size_t)(n_rows ? n_rows : 1), &N.lens)) ||
      (rc = ws_get(c, 36, (size_t)scan_blocks(n_rows) + 1, &bsum)) || (rc = ws_get(c, 4, 1, &N.err)))
    return rc;
  if (!c->h_tot) HIP_TRY(hipHostMalloc((void**)&c->h_tot, 8 * sizeof(int64_t)));
  HIP_TRY(hipMemsetAsync(N.err, 0, 4, st));
  HIP_TRY(launch_npy_len(N, c->n_cu, st));
  HIP_TRY(launch_scan_ntok(N.lens, n_rows, d_out_off, bsum, st));
  HIP_TRY(hipMemcpyAsync(&c->h_tot[6], d_out_off + n_rows, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(&c->h_tot[7], N.err, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if ((int32_t)(c->h_tot[7] & 0xFFFFFFFF)) return set_err(LDDL_EINVAL, "a row has more than kmax = %d masked positions", kmax);
  *out_nbytes = c->h_tot[6];
  if (!d_out_bytes) return 0;  // size query
  if (out_cap < c->h_tot[6])
    return set_err(LDDL_ECAPACITY, "render needs %lld bytes, out_cap %lld", (long long)c->h_tot[6], (long long)out_cap);
  if (n_rows > 0 && c->h_tot[6] > 2 * (int64_t)N.hdr_u16 * n_rows && !d_mlm_pos) return set_err(LDDL_EINVAL, "null pointer");
  N.out_off = d_out_off;
  N.out = d_out_bytes;
  HIP_TRY(launch_npy_bytes(N, c->n_cu, st));
  return 0;
}

extern "C" int lddl_render_masked(lddl_ctx* c, const uint16_t* d_ids, const int64_t* d_src, const uint16_t* d_len,
                                  const uint16_t* d_len0, int32_t segment, const int64_t* d_mlm_off,
                                  const uint16_t* d_mlm_pos, const uint16_t* d_mlm_token, int64_t row0, int64_t n_rows,
                                  int64_t* d_out_off, uint8_t* d_out_bytes, int64_t out_cap, int64_t* out_nbytes,
                                  void* stream) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  if (segment != 0 && segment != 1) return set_err(LDDL_EINVAL, "segment %d not 0 / 1", segment);
  if (row0 < 0 || n_rows < 0) return set_err(LDDL_EINVAL, "negative row range");
  if (!d_ids || !d_src || !d_len || !d_len0 || !d_mlm_off || !d_mlm_pos || !d_mlm_token || !d_out_off || !out_nbytes)
    return set_err(LDDL_EINVAL, "null pointer");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  RenderParams R{};
  R.tokens = d_ids;
  R.row_off = d_src;
  R.len0 = d_len;
  R.row0 = row0;
  R.n_rows = n_rows;
  R.segment = RENDER_SPAN;
  R.vinfo = c->d_rinfo;
  R.vpool = c->d_rpool;
  R.moff = d_mlm_off;
  R.mpos = d_mlm_pos;
  R.mtok = d_mlm_token;
  R.len0m = d_len0;
  R.mseg = segment;
  int64_t* bsum;
  int rc;
  if ((rc = ws_get(c, 35, (size_t)n_rows, &R.lens))) return rc;
  if ((rc = ws_get(c, 36, (size_t)scan_blocks(n_rows) + 1, &bsum))) return rc;
  HIP_TRY(launch_render_len(R, c->n_cu, st));
  HIP_TRY(launch_scan_ntok(R.lens, n_rows, d_out_off, bsum, st));
  HIP_TRY(hipMemcpyAsync(&c->h_tot[6], d_out_off + n_rows, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  *out_nbytes = c->h_tot[6];
  if (!d_out_bytes) return 0;
  if (out_cap < c->h_tot[6])
    return set_err(LDDL_ECAPACITY, "render needs %lld bytes, out_cap %lld", (long long)c->h_tot[6], (long long)out_cap);
  R.out_off = d_out_off;
  R.out = d_out_bytes;
  HIP_TRY(launch_render_bytes(R, c->n_cu, st));
  return 0;
}

extern "C" int lddl_row_docs(lddl_ctx* c, lddl_pack* pk, int64_t* d_out_doc, void* stream) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  lddl_pack* k = pk ? pk : &c->own;
  if (k->device != c->device) return set_err(LDDL_EINVAL, "pack result of another device");
  if (k->last_npairs < 0) return set_err(LDDL_EINVAL, "no successful lddl_pack_* call");
  if (!d_out_doc) return set_err(LDDL_EINVAL, "null pointer");
  HIP_TRY(hipSetDevice(c->device));
  const PackParams& P = k->pp;
  RowDocParams D{};
  D.pairs = P.pairs;
  D.binned = P.binned;
  D.pair_base = (const int64_t*)k->ws[15].p;
  D.fs_base = P.fs_base;
  D.sent_off = P.sent_off;
  D.doc_sent_off = P.doc_sent_off;
  D.part_doc_off = P.part_doc_off;
  D.n_part = P.n_part;
  D.n_rows = k->last_npairs;
  D.dup = P.dup;
  D.out_doc = d_out_doc;
  HIP_TRY(launch_row_docs(D, c->n_cu, (hipStream_t)stream));
  return 0;
}

// -------------------------------------------------------------- collate --
static int collate_vocab(lddl_ctx* c, CollateVocab* V) {
  if (!c->d_ctab) {
    const size_t n = c->vocab.size();
    uint32_t sz = 1024;
    while (sz < 4 * n) sz <<= 1;
    std::vector<uint2> tab(sz, make_uint2(0u, 0xFFFFFFFFu));
    for (size_t i = 0; i < n; ++i) {
      const std::string& w = c->vocab[i];
      const uint32_t h = collate_hash_host((const uint8_t*)w.data(), (int)w.size());
      for (uint32_t s = h & (sz - 1);; s = (s + 1) & (sz - 1)) {
        if (tab[s].y == 0xFFFFFFFFu) {
          tab[s] = make_uint2(h, (uint32_t)i);
          break;
        }
        if (tab[s].x == h && c->vocab[tab[s].y] == w) {  // duplicate line: last id wins
          tab[s].y = (uint32_t)i;
          break;
        }
      }
    }
    int rc;
    if ((rc = upload(&c->d_ctab, tab.data(), tab.size() * sizeof(uint2)))) return rc;
    c->ctab_mask = sz - 1;
  }
  V->slots = c->d_ctab;
  V->mask = c->ctab_mask;
  V->vinfo = c->d_rinfo;
  V->vpool = c->d_rpool;
  V->unk = (int32_t)c->special[1];
  V->cls = (int32_t)c->special[2];
  V->sep = (int32_t)c->special[3];
  V->mask_id = (int32_t)c->special[4];
  V->n_random = c->vocab_size;
  return 0;
}

extern "C" int lddl_collate_seq_len(lddl_ctx* c, const uint8_t* d_a, const int64_t* d_a_off, const uint8_t* d_b,
                                    const int64_t* d_b_off, int64_t n_rows, int32_t seq_align, int64_t* out_seq_len,
                                    void* stream) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  if (n_rows < 0 || seq_align < 1 || !out_seq_len) return set_err(LDDL_EINVAL, "bad n_rows / seq_align / out");
  if (n_rows > 0 && (!d_a || !d_a_off || !d_b || !d_b_off)) return set_err(LDDL_EINVAL, "null column pointer");
  if (n_rows == 0) return set_err(LDDL_EINVAL, "empty batch (max() of an empty sequence)");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  CollateParams P{};
  int rc;
  if ((rc = collate_vocab(c, &P.V))) return rc;
  P.a = d_a;
  P.a_off = d_a_off;
  P.b = d_b;
  P.b_off = d_b_off;
  P.n_rows = n_rows;
  if ((rc = ws_get(c, 37, 1, &P.max_len))) return rc;
  if (!c->h_tot) HIP_TRY(hipHostMalloc((void**)&c->h_tot, 8 * sizeof(int64_t)));
  HIP_TRY(hipMemsetAsync(P.max_len, 0, 4, st));
  HIP_TRY(launch_collate_len(P, c->n_cu, st));
  HIP_TRY(hipMemcpyAsync(&c->h_tot[7], P.max_len, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const int64_t m = *(const int32_t*)&c->h_tot[7];
  *out_seq_len = ((m - 1) / seq_align + 1) * seq_align;
  return 0;
}

extern "C" int lddl_collate_bert(lddl_ctx* c, const uint8_t* d_a, const int64_t* d_a_off, const uint8_t* d_b,
                                 const int64_t* d_b_off, const uint8_t* d_is_random_next, const uint8_t* d_pos,
                                 const int64_t* d_pos_off, const uint8_t* d_lab, const int64_t* d_lab_off,
                                 int64_t n_rows, int64_t seq_len, int32_t mode, int64_t ignore_index,
                                 double mlm_probability, uint64_t seed, uint64_t counter, int64_t* d_input_ids,
                                 int64_t* d_token_type_ids, int64_t* d_attention_mask, int64_t* d_labels,
                                 int64_t* d_next_sentence_labels, void* stream) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  if (n_rows < 0) return set_err(LDDL_EINVAL, "negative n_rows");
  if (mode < COLLATE_SPECIAL_MASK || mode > COLLATE_DYNAMIC) return set_err(LDDL_EINVAL, "mode %d not in 0..2", mode);
  if (seq_len < 3 || seq_len > COLLATE_MAX_LEN)
    return set_err(LDDL_ECAPACITY, "seq_len %lld not in [3, %d]", (long long)seq_len, COLLATE_MAX_LEN);
  if (ignore_index < INT32_MIN || ignore_index > INT32_MAX) return set_err(LDDL_EINVAL, "ignore_index out of int32");
  if (!(mlm_probability >= 0.0 && mlm_probability <= 1.0)) return set_err(LDDL_EINVAL, "mlm_probability not in [0, 1]");
  if (n_rows > 0 && (!d_a || !d_a_off || !d_b || !d_b_off || !d_is_random_next || !d_input_ids ||
                     !d_token_type_ids || !d_attention_mask || !d_labels || !d_next_sentence_labels))
    return set_err(LDDL_EINVAL, "null pointer");
  if (mode == COLLATE_STATIC && n_rows > 0 && (!d_pos || !d_pos_off || !d_lab || !d_lab_off))
    return set_err(LDDL_EINVAL, "static masking needs positions and labels");
  if (n_rows == 0) return 0;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  CollateParams P{};
  int rc;
  if ((rc = collate_vocab(c, &P.V))) return rc;
  P.a = d_a;
  P.a_off = d_a_off;
  P.b = d_b;
  P.b_off = d_b_off;
  P.is_random_next = d_is_random_next;
  P.pos = d_pos;
  P.pos_off = d_pos_off;
  P.lab = d_lab;
  P.lab_off = d_lab_off;
  P.n_rows = n_rows;
  P.seq_len = (int32_t)seq_len;
  P.mode = mode;
  P.ignore_index = ignore_index;
  P.mlm_probability = mlm_probability;
  P.seed = seed;
  P.counter = counter;
  P.input_ids = d_input_ids;
  P.token_type_ids = d_token_type_ids;
  P.attention_mask = d_attention_mask;
  P.labels = d_labels;
  P.next_sentence_labels = d_next_sentence_labels;
  if ((rc = ws_get(c, 39, 1, &P.err))) return rc;
  if (!c->h_tot) HIP_TRY(hipHostMalloc((void**)&c->h_tot, 8 * sizeof(int64_t)));
  HIP_TRY(hipMemsetAsync(P.err, 0, 4, st));
  HIP_TRY(launch_collate_fill(P, c->n_cu, st));
  uint32_t* h_err = (uint32_t*)&c->h_tot[7];
  HIP_TRY(hipMemcpyAsync(h_err, P.err, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const uint32_t e = *h_err;
  if (e) {
    const unsigned long long row = e >> 4;
    switch (e & 15u) {
      case CERR_LONG: return set_err(LDDL_ECAPACITY, "row %llu longer than seq_len %lld", row, (long long)seq_len);
      case CERR_POS_RANGE:
        return set_err(LDDL_EINDEX, "row %llu: masked_lm_positions index out of range for seq_len %lld", row,
                       (long long)seq_len);
      case CERR_NPY: return set_err(LDDL_EFORMAT, "row %llu: masked_lm_positions is not np.save bytes", row);
      default:
        return set_err(LDDL_EFORMAT, "row %llu: masked_lm_positions and masked_lm_labels differ in length", row);
    }
  }
  return 0;
}

extern "C" int lddl_mask_tokens(lddl_ctx* c, int64_t* d_inputs, const int64_t* d_special_tokens_mask,
                                int64_t* d_labels, int64_t n_rows, int64_t seq_len, double mlm_probability,
                                int64_t ignore_index, uint64_t seed, uint64_t counter, void* stream) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  if (n_rows < 0 || seq_len < 0 || seq_len >= (1 << 20)) return set_err(LDDL_EINVAL, "bad shape");
  if (!(mlm_probability >= 0.0 && mlm_probability <= 1.0)) return set_err(LDDL_EINVAL, "mlm_probability not in [0, 1]");
  if (n_rows * seq_len > 0 && (!d_inputs || !d_special_tokens_mask || !d_labels))
    return set_err(LDDL_EINVAL, "null pointer");
  HIP_TRY(hipSetDevice(c->device));
  MaskParams M{};
  M.inputs = d_inputs;
  M.special = d_special_tokens_mask;
  M.labels = d_labels;
  M.n_rows = n_rows;
  M.seq_len = (int32_t)seq_len;
  M.mask_id = (int32_t)c->special[4];
  M.n_random = c->vocab_size;
  M.ignore_index = ignore_index;
  M.mlm_probability = mlm_probability;
  M.seed = seed;
  M.counter = counter;
  HIP_TRY(launch_mask_tokens(M, c->n_cu, (hipStream_t)stream));
  return 0;
}
