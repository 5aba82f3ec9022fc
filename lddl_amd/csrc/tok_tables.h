// Host-side tokenizer tables: the unicode table file (tools/gen_unicode_table.py)
// and a vocab.txt turned into the arrays TokParams points at.  Host C++ only
// (no HIP calls): capi.hip uploads the results; tests/host_serial.cpp runs the
// serial tokenizer path (tokenize_serial.h) over them on the host under
// AddressSanitizer.  Reference: the vocab / BertNormalizer of the tokenizer
// that lddl/dask/bert/pretrain.py:79-80 calls.
#pragma once
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lddl_amd.h"
#include "common.h"
#include "tokenize.h"

namespace lddl {

struct UniTables {
  std::vector<uint16_t> top;     // [0x1100] page of each 256-code-point block
  std::vector<uint32_t> pages;   // [npages * 256] entries (common.h ent_*)
  std::vector<uint32_t> multi;   // [nmulti * 4] multi-char expansions
  std::vector<uint32_t> bmp;     // [0x10000] flattened BMP entries
  std::vector<uint32_t> xmap;    // [0x110000] the split scan's fast exception entries
  bool scan_ok = false;          // the ASCII page fits the split scan's per-byte class table
  // lane tokenizer (tokenize_lane.hip): per byte, its normalised byte | class << 8 (LANE_C*);
  // lane_ok: no code point normalises to more chars than its UTF-8 bytes, so a
  // sentence never has more tokens than bytes (its ids are staged at its byte offset)
  std::vector<uint16_t> lane_ctab;
  bool lane_ok = false;
};



struct VocabTables {
  std::vector<std::string> vocab;
  uint32_t special[5] = {0, 0, 0, 0, 0};  // [PAD] [UNK] [CLS] [SEP] [MASK]
  uint32_t maxb[2] = {0, 0};              // longest key without / with "##"
  std::vector<uint8_t> pool;              // (cont, bytes) keys, each 4-aligned
  std::vector<uint32_t> voff;             // [V] key offset in pool
  std::vector<uint4> slots;               // open-addressing slots (serial path)
  uint32_t slot_mask = 0;
  std::vector<uint32_t> bloom;            // [BLOOM_WORDS] over the slot keys
  std::vector<uint32_t> vt;               // v4 buckets: two 32-B slots each
  uint32_t vt_mask = 0;
  std::vector<uint32_t> vbloom;           // [BLOOM_WORDS] over the v4 keys + extension keys
  std::vector<uint32_t> st;               // the scan's whole-word table: 32-B slots, two choices per key
  uint32_t st_mask = 0;
  std::vector<uint8_t> rpool;             // vocab entries verbatim, 4-aligned (rendering)
  std::vector<uint32_t> rinfo;            // [V] offset << 8 | length into rpool
  std::vector<uint2> trie;                // lane tokenizer's double-array trie (trie_* below)
  uint32_t trie_base[2] = {0, 0};         // children offsets of the two roots (whole word, "##")
};

// ---- double-array trie of the vocab keys (layout: common.h trie_*) -------
// keys[i] = (cont, bytes) of vocab id i (empty: none); the last duplicate wins.
// Returns false when the array would pass 2^20 entries.
inline bool build_trie(const std::vector<std::string>& vocab, std::vector<uint2>& da, uint32_t base_out[2]) {
  struct Node {
    std::vector<std::pair<uint8_t, uint32_t>> kids;  // byte -> node
    int32_t id = -1;
  };
  std::vector<Node> nodes(2);
  for (size_t i = 0; i < vocab.size(); ++i) {
    const std::string& w = vocab[i];
    const uint32_t cont = (w.size() >= 2 && w[0] == '#' && w[1] == '#') ? 1u : 0u;
    if (w.size() == 2 * cont) continue;  // "" / "##": no key
    uint32_t n = cont;
    for (size_t k = 2 * cont; k < w.size(); ++k) {
      const uint8_t c = (uint8_t)w[k];
      uint32_t nx = 0;
      for (auto& kc : nodes[n].kids)
        if (kc.first == c) nx = kc.second;
      if (!nx) {
        nx = (uint32_t)nodes.size();
        nodes[n].kids.push_back({c, nx});
        nodes.emplace_back();
      }
      n = nx;
    }
    nodes[n].id = (int32_t)i;
  }
  // place breadth-first: slot[node], base[node]; first fit over a used map,
  // the candidates for a node's first child walked over free slots only
  // (nxt: the next free slot at or after p, path-halved)
  const uint32_t CAPS = 1u << 20;
  std::vector<uint32_t> slot(nodes.size(), 0), base(nodes.size(), 0);
  std::vector<uint8_t> used(CAPS + 256, 0);
  std::vector<uint32_t> nxt(CAPS + 257);
  for (uint32_t p = 0; p < nxt.size(); ++p) nxt[p] = p;
  auto find = [&](uint32_t p) {
    while (nxt[p] != p) {
      nxt[p] = nxt[nxt[p]];
      p = nxt[p];
    }
    return p;
  };
  auto take = [&](uint32_t p) {
    used[p] = 1;
    nxt[p] = p + 1;
  };
  take(0);
  take(1);
  slot[0] = 0;
  slot[1] = 1;
  std::vector<uint32_t> order = {0, 1};
  uint32_t top = 2;
  for (size_t qi = 0; qi < order.size(); ++qi) {
    Node& nd = nodes[order[qi]];
    if (nd.kids.empty()) continue;
    std::sort(nd.kids.begin(), nd.kids.end());
    const uint32_t c0 = nd.kids[0].first;
    uint32_t b = 0;
    for (uint32_t p = find(c0);; p = find(p + 1)) {  // p: a free slot for the first child
      b = p - c0;
      if (b + 256 >= CAPS) return false;
      bool fit = true;
      for (auto& kc : nd.kids)
        if (used[b + kc.first]) { fit = false; break; }
      if (fit) break;
    }
    base[order[qi]] = b;
    for (auto& kc : nd.kids) {
      take(b + kc.first);
      slot[kc.second] = b + kc.first;
      order.push_back(kc.second);
      if (b + kc.first + 1 > top) top = b + kc.first + 1;
    }
  }
  uint32_t maxb = 0;
  for (uint32_t b : base) maxb = b > maxb ? b : maxb;
  const size_t size = std::max<size_t>(top, (size_t)maxb + 256) + 1;
  if (size >= TRIE_EMPTY) return false;
  da.assign(size, make_uint2(TRIE_EMPTY, 0u));
  for (size_t i = 0; i < nodes.size(); ++i) {
    const int32_t id = nodes[i].id < 0 ? 0 : nodes[i].id;
    uint2 e;
    e.x = TRIE_EMPTY | ((uint32_t)id & 0xFFFu) << 20;
    e.y = base[i] | (((uint32_t)id >> 12) & 0xFu) << 20 | (nodes[i].id >= 0 ? 0x80000000u : 0u);
    da[slot[i]] = e;
  }
  for (size_t i = 0; i < nodes.size(); ++i)
    for (auto& kc : nodes[i].kids) da[slot[kc.second]].x = (da[slot[kc.second]].x & ~0xFFFFFu) | slot[i];
  base_out[0] = base[0];
  base_out[1] = base[1];
  return true;
}

// Returns 0, or an LDDL_E* code with the reason in err.
inline int build_uni_tables(const char* path, UniTables& T, std::string& err) {
  FILE* f = fopen(path, "rb");
  if (!f) { err = std::string("cannot open unicode table ") + path; return LDDL_EIO; }
  char magic[8];
  uint32_t hdr[3];
  T.top.assign(0x1100, 0);
  if (fread(magic, 1, 8, f) != 8 || memcmp(magic, "LDDLUNI1", 8) != 0 || fread(hdr, 4, 3, f) != 3) {
    fclose(f);
    err = std::string("bad unicode table header in ") + path;
    return LDDL_EFORMAT;
  }
  T.pages.assign((size_t)hdr[0] * 256, 0);
  T.multi.assign((size_t)hdr[1] * 4, 0);
  const bool ok = fread(T.top.data(), 2, T.top.size(), f) == T.top.size() &&
                  fread(T.pages.data(), 4, T.pages.size(), f) == T.pages.size() &&
                  fread(T.multi.data(), 4, T.multi.size(), f) == T.multi.size();
  fclose(f);
  if (!ok) { err = std::string("truncated unicode table ") + path; return LDDL_EFORMAT; }
  for (size_t i = 0; i < T.top.size(); ++i)
    if (T.top[i] >= hdr[0]) { err = "unicode table page index out of range"; return LDDL_EFORMAT; }
  // the kernels assume multi-char expansions are plain word chars (checked)
  for (size_t i = 0; i < hdr[1]; ++i) {
    const uint32_t n = T.multi[i * 4];
    if (n < 2 || n > 3) { err = "unicode table multi entry " + std::to_string(i) + " has " + std::to_string(n) + " chars"; return LDDL_EFORMAT; }
    for (uint32_t k = 0; k < n; ++k)
      if (ent_cls(T.multi[i * 4 + 1 + k]) != CLS_OTHER) {
        err = "unicode table multi entry " + std::to_string(i) + " has a non-word char";
        return LDDL_EFORMAT;
      }
  }
  // the split scan (tokenize_split.hip) derives its per-byte class table from the ASCII page: it
  // needs rank-0, single-char entries whose only mapping is A-Z -> a-z
  T.scan_ok = true;
  for (uint32_t b = 0; b < 128; ++b) {
    const uint32_t e = T.pages[(size_t)T.top[0] * 256 + b];
    const uint32_t kind = ent_kind(e), cls = ent_cls(e);
    if (ent_rank(e) != 0 || kind == KIND_MULTI) T.scan_ok = false;
    if (kind == KIND_MAP && cls == CLS_ISOLATE) T.scan_ok = false;
    if (kind == KIND_MAP && cls == CLS_OTHER && !(b >= 'A' && b <= 'Z' && ent_payload(e) == b + 32)) T.scan_ok = false;
  }
  if (ent_cls(T.pages[(size_t)T.top[0] * 256 + '[']) != CLS_ISOLATE) T.scan_ok = false;
  // the lane tokenizer's byte classes: an ASCII word char (normalised byte
  // below 0x80), an ASCII isolate, space, drop, '[', else the slow path
  T.lane_ctab.assign(256, (uint16_t)(LANE_CNA << 8));
  T.lane_ok = true;
  for (uint32_t b = 0; b < 128; ++b) {
    const uint32_t e = T.pages[(size_t)T.top[0] * 256 + b];
    const uint32_t kind = ent_kind(e), cls = ent_cls(e), out = kind == KIND_IDENT ? b : ent_payload(e);
    uint32_t c = LANE_CNA;
    if (ent_rank(e) != 0 || kind == KIND_MULTI) c = LANE_CNA;
    else if (kind == KIND_DROP_T || kind == KIND_DROP_D) c = LANE_CDR;
    else if (cls == CLS_SPACE) c = LANE_CSP;
    else if (out >= 0x80) c = LANE_CNA;
    else if (cls == CLS_ISOLATE) c = b == '[' ? (out == '[' ? LANE_CLB : LANE_CNA) : LANE_CI;
    else c = LANE_CW;
    if (b == '[' && c != LANE_CLB) c = LANE_CNA;  // (specials are matched on the raw byte)
    T.lane_ctab[b] = (uint16_t)((c << 8) | (out < 0x80 ? out : 0u));
  }
  for (uint32_t cp = 0x80; cp < 0x110000; ++cp) {
    const uint32_t e = T.pages[(size_t)T.top[cp >> 8] * 256 + (cp & 255)];
    if (ent_kind(e) == KIND_MULTI && T.multi[(size_t)ent_payload(e) * 4] > (cp < 0x800 ? 2u : cp < 0x10000 ? 3u : 4u))
      T.lane_ok = false;
  }
  // the BMP flattened (256 KiB, L2-resident): one load per code point < U+10000
  T.bmp.assign(0x10000, 0);
  for (uint32_t cp = 0; cp < 0x10000; ++cp) T.bmp[cp] = T.pages[(size_t)T.top[cp >> 8] * 256 + (cp & 255)];
  // the scan's fast exception entries (4.25 MiB, U+0000..U+10FFFF): what the
  // full path would do with a code point, precomputed -- its pre-tokenizer
  // action and, for a single-char mapping, the replacement's UTF-8 bytes;
  // SLOW where the full path is needed (multi-char expansion, canonical
  // reordering rank, a 4-byte replacement)
  T.xmap.assign(0x110000, 0);
  for (uint32_t cp = 0; cp < 0x110000; ++cp) {
    const uint32_t e = T.pages[(size_t)T.top[cp >> 8] * 256 + (cp & 255)];
    const uint32_t kind = ent_kind(e), cls = ent_cls(e), pay = ent_payload(e);
    uint32_t x = 0;
    if (ent_rank(e) != 0) {
      x = 0x80000000u;
    } else if (kind == KIND_DROP_T || kind == KIND_DROP_D) {
      x = 3u << 27;
    } else if (cls == CLS_SPACE) {
      x = 1u << 27;
    } else {
      x = (cls == CLS_ISOLATE ? 2u : 0u) << 27;
      if (kind == KIND_MULTI || (kind != KIND_IDENT && pay >= 0x10000)) {
        x = 0x80000000u;
      } else if (kind != KIND_IDENT) {
        uint32_t b = 0, t;
        if (pay < 0x80) { b = pay; t = 1; }
        else if (pay < 0x800) { b = (0xC0 | (pay >> 6)) | ((0x80 | (pay & 0x3F)) << 8); t = 2; }
        else { b = (0xE0 | (pay >> 12)) | ((0x80 | ((pay >> 6) & 0x3F)) << 8) | ((0x80 | (pay & 0x3F)) << 16); t = 3; }
        x |= 0x20000000u | (t << 24) | b;
      }
    }
    T.xmap[cp] = x;
  }
  return 0;
}

// with_trie: also the double-array trie (the lane tokenizer and the trie
// WordPiece read it; the default tok5 path does not)
inline int build_vocab_tables(const char* path, VocabTables& V, std::string& err, bool with_trie = true) {
  FILE* f = fopen(path, "rb");
  if (!f) { err = std::string("cannot open vocab ") + path; return LDDL_EIO; }
  std::string cur;
  int ch;
  while ((ch = fgetc(f)) != EOF) {
    if (ch == '\n') {
      while (!cur.empty() && cur.back() == '\r') cur.pop_back();
      V.vocab.push_back(cur);
      cur.clear();
    } else {
      cur.push_back((char)ch);
    }
  }
  if (!cur.empty()) V.vocab.push_back(cur);
  fclose(f);
  const size_t n = V.vocab.size();
  if (n == 0 || n > 65536) { err = "vocab size " + std::to_string(n) + " not in [1, 65536]"; return LDDL_EFORMAT; }
  const char* sp[5] = {"[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"};
  for (int k = 0; k < 5; ++k) {
    int found = -1;
    for (size_t i = 0; i < n; ++i)
      if (V.vocab[i] == sp[k]) found = (int)i;  // last occurrence wins
    if (found < 0) { err = std::string("vocab ") + path + " lacks " + sp[k]; return LDDL_EFORMAT; }
    V.special[k] = (uint32_t)found;
  }
  // pool of (cont, bytes) keys; "##x" -> cont=1 "x"; every key 4-aligned
  std::vector<uint32_t> vlen(n), vcont(n);
  V.voff.assign(n, 0);
  V.pool.clear();
  for (size_t i = 0; i < n; ++i) {
    const std::string& w = V.vocab[i];
    const uint32_t cont = (w.size() >= 2 && w[0] == '#' && w[1] == '#') ? 1u : 0u;
    const char* s = w.data() + 2 * cont;
    const uint32_t len = (uint32_t)w.size() - 2 * cont;
    if (len > 255) { err = "vocab entry " + std::to_string(i) + " longer than 255 bytes"; return LDDL_EFORMAT; }
    V.voff[i] = (uint32_t)V.pool.size();
    vlen[i] = len;
    vcont[i] = cont;
    V.pool.insert(V.pool.end(), s, s + len);
    V.pool.resize((V.pool.size() + 3) & ~(size_t)3, 0);
    if (len > V.maxb[cont]) V.maxb[cont] = len;
  }
  V.pool.resize(V.pool.size() + 16, 0);
  const std::vector<uint8_t>& pool = V.pool;
  auto same = [&](size_t a, size_t b) {
    return vlen[a] == vlen[b] && vcont[a] == vcont[b] && memcmp(&pool[V.voff[a]], &pool[V.voff[b]], vlen[b]) == 0;
  };
  uint32_t cap = 1;
  while (cap < n * 2) cap <<= 1;
  V.slots.assign(cap, make_uint4(0, 0, 0, 0));
  for (size_t i = 0; i < n; ++i) {
    if (vlen[i] == 0) continue;  // "##" alone: unreachable
    uint64_t h = 0;
    for (uint32_t k = 0; k < vlen[i]; ++k) h = hash_push(h, pool[V.voff[i] + k]);
    const uint64_t key = hash_key(h, vlen[i], vcont[i]);
    uint32_t idx = (uint32_t)key & (cap - 1);
    const uint32_t fp = (uint32_t)(key >> 32);
    uint32_t pre[2] = {0, 0};
    memcpy(pre, &pool[V.voff[i]], vlen[i] < 8 ? vlen[i] : 8);
    for (;;) {
      uint4& s = V.slots[idx];
      if (!(s.y & 0x80000000u)) { s = make_uint4(fp, slot_info((uint32_t)i, vlen[i], vcont[i]), pre[0], pre[1]); break; }
      if (same(s.y & 0xFFFFu, i)) {
        s.y = slot_info((uint32_t)i, vlen[i], vcont[i]);  // duplicate line: last id wins
        break;
      }
      idx = (idx + 1) & (cap - 1);
    }
  }
  V.slot_mask = cap - 1;
  // blocked Bloom filter over the same keys: word = key bits 40..52, two bit
  // positions from key bits 0..9.  A clear bit proves absence (exact negative).
  V.bloom.assign(BLOOM_WORDS, 0);
  for (size_t i = 0; i < n; ++i) {
    if (vlen[i] == 0) continue;
    uint64_t h = 0;
    for (uint32_t k = 0; k < vlen[i]; ++k) h = hash_push(h, pool[V.voff[i] + k]);
    const uint64_t key = hash_key(h, vlen[i], vcont[i]);
    V.bloom[(uint32_t)(key >> 40) & (BLOOM_WORDS - 1)] |= (1u << (key & 31)) | (1u << ((key >> 5) & 31));
  }
  // v4 table: buckets of two 32-B slots, linear probing over buckets; Bloom
  // filter over the same hashes (common.h vhash)
  // The scan's whole-word probe reads only slot 0 of a word's home bucket
  // (tokenize_split.hip): a vocab word displaced from it is not found there
  // and costs a WordPiece record.  So the buckets are >= 16V (load <= 1/32;
  // simulated on the synthetic Wikipedia text: 0.3 % of the whole-word unit
  // occurrences off slot 0, against 3-6 % at 2V; the table is read at a few
  // thousand hot lines whatever its size) and every whole-word key (cont = 0,
  // in vocab order: the frequent words first) is inserted before the "##"
  // pieces, which the scan never looks up.
  uint32_t nbk = 1;
  while (nbk < 16 * n) nbk <<= 1;
  V.vt.assign((size_t)nbk * 16, 0u);
  V.vbloom.assign(BLOOM_WORDS, 0u);
  std::vector<size_t> order;
  order.reserve(n);
  for (int pass = 0; pass < 2; ++pass)
    for (size_t i = 0; i < n; ++i)
      if (vlen[i] != 0 && (uint32_t)vcont[i] == (uint32_t)pass) order.push_back(i);
  for (size_t i : order) {
    uint32_t d[VKEY_DW] = {0, 0, 0, 0, 0, 0};
    memcpy(d, &pool[V.voff[i]], vlen[i] < 24 ? vlen[i] : 24);
    const uint32_t h = vhash(d, vlen[i], vcont[i]), bk = vbkey_of(d, vlen[i], vcont[i]);
    V.vbloom[vbloom_word(bk)] |= vbloom_bits(bk);
    {  // extension keys of its 4-, 8-, .. 24-byte prefixes shorter than it
      uint32_t hp = VSEED;
      for (uint32_t j = 0; j < VKEY_DW && 4 * (j + 1) < vlen[i]; ++j) {
        hp = vmix(hp, d[j]);
        const uint32_t ek = vbkey_ext(hp, 4 * (j + 1), vcont[i]);
        V.vbloom[vbloom_word(ek)] |= vbloom_bits(ek);
      }
    }
    bool done = false;
    for (uint32_t b = h & (nbk - 1); !done; b = (b + 1) & (nbk - 1)) {
      for (int sl = 0; sl < 2 && !done; ++sl) {
        uint32_t* s = &V.vt[((size_t)b * 2 + sl) * 8];
        if (s[6] != 0 && !same(s[6] & 0xFFFFu, i)) continue;  // occupied by another key
        memcpy(s, d, sizeof d);  // empty slot, or a duplicate line: last id wins
        s[6] = slot_info((uint32_t)i, vlen[i], vcont[i]);
        s[7] = V.voff[i];
        done = true;
      }
    }
  }
  V.vt_mask = nbk - 1;
  // the scan's whole-word table: every whole-word key of <= 24 bytes (the
  // keys the scan probes) in one of its two slots (st_second), placed by
  // cuckoo moves, >= 2.5 slots per key: 64 K slots (2 MB) for BERT, so the
  // probes of words outside the vocab hit L2 instead of random lines of the
  // 32 MB bucket table.  A duplicate line: the last id wins, as in vt.
  {
    std::vector<size_t> keys;
    for (size_t i : order)
      if (vcont[i] == 0 && vlen[i] <= 24) keys.push_back(i);
    uint32_t ns = 1024;
    while (ns < keys.size() * 5 / 2) ns <<= 1;
    auto key_of = [&](size_t i, uint32_t* d) {
      for (int q = 0; q < VKEY_DW; ++q) d[q] = 0;
      memcpy(d, &pool[V.voff[i]], vlen[i]);
    };
    for (;;) {
      V.st.assign((size_t)ns * 8, 0u);
      const uint32_t m = ns - 1;
      bool ok = true;
      for (size_t i : keys) {
        uint32_t e[8];
        key_of(i, e);
        e[6] = slot_info((uint32_t)i, vlen[i], 0);
        e[7] = V.voff[i];
        const uint32_t h = vhash(e, vlen[i], 0);
        const uint32_t p1 = h & m, p2 = st_second(h) & m;
        bool dup = false;
        for (uint32_t p : {p1, p2}) {
          uint32_t* s = &V.st[(size_t)p * 8];
          if (s[6] != 0 && same(s[6] & 0xFFFFu, i)) {
            s[6] = e[6];  // (last id wins)
            dup = true;
            break;
          }
        }
        if (dup) continue;
        uint32_t pos = V.st[(size_t)p1 * 8 + 6] == 0 ? p1 : p2;
        bool placed = false;
        for (int kick = 0; kick < 1000 && !placed; ++kick) {
          uint32_t* s = &V.st[(size_t)pos * 8];
          if (s[6] == 0) {
            memcpy(s, e, sizeof e);
            placed = true;
            break;
          }
          uint32_t out[8];
          memcpy(out, s, sizeof out);
          memcpy(s, e, sizeof e);
          memcpy(e, out, sizeof out);
          const uint32_t hl = vhash(e, (e[6] >> 16) & 0xFFu, 0);
          pos = (pos == (hl & m)) ? (st_second(hl) & m) : (hl & m);
        }
        if (!placed) {
          ok = false;
          break;
        }
      }
      if (ok) break;
      ns <<= 1;  // (a cycle: a larger table)
    }
    V.st_mask = ns - 1;
  }
  // rendering tables: the vocab entries verbatim (pretrain.py:348-353 joins them)
  V.rpool.clear();
  V.rinfo.assign(n, 0);
  for (size_t i = 0; i < n; ++i) {
    const std::string& w = V.vocab[i];
    if (V.rpool.size() >= (1u << 24)) { err = "vocab text larger than 16 MiB"; return LDDL_EFORMAT; }
    V.rinfo[i] = (uint32_t)V.rpool.size() << 8 | (uint32_t)w.size();  // size <= 255, checked above
    V.rpool.insert(V.rpool.end(), w.begin(), w.end());
    V.rpool.resize((V.rpool.size() + 3) & ~(size_t)3, 0);
  }
  V.rpool.resize(V.rpool.size() + 16, 0);
  if (with_trie && !build_trie(V.vocab, V.trie, V.trie_base)) V.trie.clear();  // (the lane tokenizer then stays off)
  return 0;
}

}  // namespace lddl
