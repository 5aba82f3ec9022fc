// C-ABI of libldl_amd.so: the drop-in boundary (declared in include/lddl_amd.h).
// Plain pointers and sizes only; device pointers come from the caller
// (torch tensors via data_ptr(), or hipMalloc).  Every entry point returns 0
// on success and a negative LDDL_E* code on failure; the message is kept in
// a thread-local buffer readable with lddl_last_error().  Nothing aborts.
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/lddl_amd.h"
#include "common.h"
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

struct lddl_ctx {
  int device = 0;
  int n_cu = 0;
  int vocab_size = 0;
  uint32_t special[5] = {0, 0, 0, 0, 0};
  std::vector<std::string> vocab;  // host copy (for rendering / tests)
  // device tables
  uint16_t* d_top = nullptr;
  uint32_t* d_pages = nullptr;
  uint4* d_multi = nullptr;
  uint2* d_slots = nullptr;
  uint32_t slot_mask = 0;
  uint8_t* d_pool = nullptr;
  uint32_t* d_voff = nullptr;
  uint32_t maxb[2] = {0, 0};
  // scratch
  int tok_grid = 0;
  uint8_t* d_ovf = nullptr;
  uint32_t* d_counter = nullptr;
};

extern "C" const char* lddl_last_error(void) { return g_err; }

static void free_ctx(lddl_ctx* c) {
  if (!c) return;
  (void)hipFree(c->d_top);
  (void)hipFree(c->d_pages);
  (void)hipFree(c->d_multi);
  (void)hipFree(c->d_slots);
  (void)hipFree(c->d_pool);
  (void)hipFree(c->d_voff);
  (void)hipFree(c->d_ovf);
  (void)hipFree(c->d_counter);
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
  FILE* f = fopen(path, "rb");
  if (!f) return set_err(LDDL_EIO, "cannot open unicode table %s", path);
  char magic[8];
  uint32_t hdr[3];
  std::vector<uint16_t> top(0x1100);
  if (fread(magic, 1, 8, f) != 8 || memcmp(magic, "LDDLUNI1", 8) != 0 || fread(hdr, 4, 3, f) != 3) {
    fclose(f);
    return set_err(LDDL_EFORMAT, "bad unicode table header in %s", path);
  }
  std::vector<uint32_t> pages((size_t)hdr[0] * 256);
  std::vector<uint32_t> multi((size_t)hdr[1] * 4);
  bool ok = fread(top.data(), 2, top.size(), f) == top.size() &&
            fread(pages.data(), 4, pages.size(), f) == pages.size() &&
            fread(multi.data(), 4, multi.size(), f) == multi.size();
  fclose(f);
  if (!ok) return set_err(LDDL_EFORMAT, "truncated unicode table %s", path);
  for (size_t i = 0; i < top.size(); ++i)
    if (top[i] >= hdr[0]) return set_err(LDDL_EFORMAT, "unicode table page index out of range");
  // the kernel assumes multi-char expansions are plain word chars (checked)
  for (size_t i = 0; i < hdr[1]; ++i) {
    uint32_t n = multi[i * 4];
    if (n < 2 || n > 3) return set_err(LDDL_EFORMAT, "unicode table multi entry %zu has %u chars", i, n);
    for (uint32_t k = 0; k < n; ++k)
      if (ent_cls(multi[i * 4 + 1 + k]) != CLS_OTHER)
        return set_err(LDDL_EFORMAT, "unicode table multi entry %zu has a non-word char", i);
  }
  int rc;
  if ((rc = upload(&c->d_top, top.data(), top.size() * 2))) return rc;
  if ((rc = upload(&c->d_pages, pages.data(), pages.size() * 4))) return rc;
  if ((rc = upload(&c->d_multi, multi.data(), multi.size() * 4))) return rc;
  return 0;
}

static int load_vocab(lddl_ctx* c, const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) return set_err(LDDL_EIO, "cannot open vocab %s", path);
  std::string cur;
  int ch;
  while ((ch = fgetc(f)) != EOF) {
    if (ch == '\n') {
      while (!cur.empty() && cur.back() == '\r') cur.pop_back();
      c->vocab.push_back(cur);
      cur.clear();
    } else {
      cur.push_back((char)ch);
    }
  }
  if (!cur.empty()) c->vocab.push_back(cur);
  fclose(f);
  const size_t V = c->vocab.size();
  if (V == 0 || V > 65536) return set_err(LDDL_EFORMAT, "vocab size %zu not in [1, 65536]", V);
  c->vocab_size = (int)V;
  const char* sp[5] = {"[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"};
  for (int k = 0; k < 5; ++k) {
    int found = -1;
    for (size_t i = 0; i < V; ++i)
      if (c->vocab[i] == sp[k]) found = (int)i;  // last occurrence wins
    if (found < 0) return set_err(LDDL_EFORMAT, "vocab %s lacks %s", path, sp[k]);
    c->special[k] = (uint32_t)found;
  }
  // pool of (cont, bytes) keys; "##x" -> cont=1 "x"
  std::vector<uint8_t> pool;
  std::vector<uint32_t> voff(V), vlen(V), vcont(V);
  for (size_t i = 0; i < V; ++i) {
    const std::string& w = c->vocab[i];
    uint32_t cont = (w.size() >= 2 && w[0] == '#' && w[1] == '#') ? 1u : 0u;
    const char* s = w.data() + 2 * cont;
    uint32_t n = (uint32_t)w.size() - 2 * cont;
    if (n > 255) return set_err(LDDL_EFORMAT, "vocab entry %zu longer than 255 bytes", i);
    voff[i] = (uint32_t)pool.size();
    vlen[i] = n;
    vcont[i] = cont;
    pool.insert(pool.end(), s, s + n);
    if (n > c->maxb[cont]) c->maxb[cont] = n;
  }
  pool.resize(pool.size() + 16, 0);
  uint32_t cap = 1;
  while (cap < V * 5 / 2) cap <<= 1;
  std::vector<uint2> slots(cap, make_uint2(0, 0));
  for (size_t i = 0; i < V; ++i) {
    if (vlen[i] == 0) continue;  // "##" alone: unreachable
    uint64_t h = 0;
    for (uint32_t k = 0; k < vlen[i]; ++k) h = hash_push(h, pool[voff[i] + k]);
    uint64_t key = hash_key(h, vlen[i], vcont[i]);
    uint32_t idx = (uint32_t)key & (cap - 1), fp = (uint32_t)(key >> 32);
    for (;;) {
      uint2& s = slots[idx];
      if (!(s.y & 0x80000000u)) { s = make_uint2(fp, slot_info((uint32_t)i, vlen[i], vcont[i])); break; }
      uint32_t j = s.y & 0xFFFFu;
      if (vlen[j] == vlen[i] && vcont[j] == vcont[i] && memcmp(&pool[voff[j]], &pool[voff[i]], vlen[i]) == 0) {
        s.y = slot_info((uint32_t)i, vlen[i], vcont[i]);  // duplicate line: last id wins
        break;
      }
      idx = (idx + 1) & (cap - 1);
    }
  }
  c->slot_mask = cap - 1;
  int rc;
  if ((rc = upload(&c->d_slots, slots.data(), slots.size() * sizeof(uint2)))) return rc;
  if ((rc = upload(&c->d_pool, pool.data(), pool.size()))) return rc;
  if ((rc = upload(&c->d_voff, voff.data(), voff.size() * 4))) return rc;
  return 0;
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
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, tokenize_kernel_ptr(), 256, 0) != hipSuccess || per_cu < 1)
    per_cu = 4;
  c->tok_grid = c->n_cu * per_cu;
  if (hipMalloc((void**)&c->d_ovf, (size_t)c->tok_grid * 256 * WB_OVF) != hipSuccess ||
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

extern "C" int lddl_tokenize(lddl_ctx* c, const uint8_t* d_bytes, const int64_t* d_sent_off, int64_t n_sent,
                             int32_t max_tok, uint16_t* d_out_ids, int32_t* d_out_ntok, void* stream) {
  if (!c) return set_err(LDDL_EINVAL, "null ctx");
  if (n_sent < 0 || max_tok < 1) return set_err(LDDL_EINVAL, "n_sent %lld max_tok %d", (long long)n_sent, max_tok);
  if (n_sent == 0) return 0;
  if (!d_bytes || !d_sent_off || !d_out_ids || !d_out_ntok) return set_err(LDDL_EINVAL, "null device pointer");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  TokParams P{};
  P.bytes = d_bytes;
  P.sent_off = d_sent_off;
  P.n_sent = n_sent;
  P.max_tok = max_tok;
  P.chunk = 256;
  P.out_ids = d_out_ids;
  P.out_ntok = d_out_ntok;
  P.top = c->d_top;
  P.pages = c->d_pages;
  P.multi = c->d_multi;
  P.slots = c->d_slots;
  P.slot_mask = c->slot_mask;
  P.pool = c->d_pool;
  P.voff = c->d_voff;
  P.maxb[0] = c->maxb[0];
  P.maxb[1] = c->maxb[1];
  for (int k = 0; k < 5; ++k) P.special[k] = c->special[k];
  P.unk = c->special[1];
  P.ovf = c->d_ovf;
  P.work_counter = c->d_counter;
  HIP_TRY(hipMemsetAsync(c->d_counter, 0, 64, st));
  const int64_t chunks = (n_sent + P.chunk - 1) / P.chunk;
  const int64_t waves = chunks;
  int grid = (int)((waves + 3) / 4);
  if (grid > c->tok_grid) grid = c->tok_grid;
  HIP_TRY(launch_tokenize(P, grid, st));
  return 0;
}
