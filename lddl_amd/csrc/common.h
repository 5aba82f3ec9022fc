// Shared host/device definitions for the lddl_amd HIP path (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LDDL_HD __host__ __device__ __forceinline__

namespace lddl {

// ---- Unicode table entry layout (tools/gen_unicode_table.py) -------------
// bits 0-20 payload (mapped code point / multi index), 21-23 canonical
// reordering rank (0 = starter), 24-25 pre-tokenizer class, 26-28 kind.
enum : uint32_t { KIND_IDENT = 0, KIND_MAP = 1, KIND_DROP_T = 2, KIND_DROP_D = 3, KIND_MULTI = 4 };
enum : uint32_t { CLS_OTHER = 0, CLS_SPACE = 1, CLS_ISOLATE = 2 };

LDDL_HD uint32_t ent_kind(uint32_t e) { return e >> 26; }
LDDL_HD uint32_t ent_cls(uint32_t e) { return (e >> 24) & 3u; }
LDDL_HD uint32_t ent_rank(uint32_t e) { return (e >> 21) & 7u; }
LDDL_HD uint32_t ent_payload(uint32_t e) { return e & 0x1FFFFFu; }

// ---- vocab hash ------------------------------------------------------------
// Polynomial hash over the bytes of a candidate piece (without "##"), so a
// candidate can be shrunk by one byte in O(1): H' = (H - (b+1)) * P^-1.
constexpr uint64_t HASH_P = 0x100000001B3ULL;

constexpr uint64_t inv64(uint64_t a) {
  uint64_t x = a;  // Newton: x = x * (2 - a*x), 6 steps give 64 bits
  for (int i = 0; i < 6; ++i) x *= 2 - a * x;
  return x;
}
constexpr uint64_t HASH_PINV = inv64(HASH_P);
static_assert(HASH_P * HASH_PINV == 1ULL, "inverse");

LDDL_HD uint64_t hash_push(uint64_t h, uint32_t b) { return h * HASH_P + (uint64_t)(b + 1); }
LDDL_HD uint64_t hash_pop(uint64_t h, uint32_t b) { return (h - (uint64_t)(b + 1)) * HASH_PINV; }

LDDL_HD uint64_t hash_key(uint64_t h, uint32_t len, uint32_t cont) {
  uint64_t x = h ^ ((uint64_t)len << 56) ^ (cont ? 0x9E3779B97F4A7C15ULL : 0ULL);
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ULL;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBULL;
  x ^= x >> 31;
  return x;
}

// vocab hash slot (uint4): x = 32-bit fingerprint, y = info, z/w = the
// first 8 bytes of the key (zero padded) -- keys of <= 8 bytes verify from
// the slot alone; longer keys compare the rest against the 4-aligned pool.
// slot.y layout: id (16) | len (8) << 16 | cont << 24 | valid << 31
LDDL_HD uint32_t slot_info(uint32_t id, uint32_t len, uint32_t cont) {
  return id | (len << 16) | (cont << 24) | 0x80000000u;
}

// ---- vocab table (tokenize_split.hip, tokenize_serial.h) -----------------------------------
// A candidate piece is hashed from its first 24 bytes held as six
// little-endian dwords (bytes >= len zero), its byte length and the "##"
// flag.  The table is an array of 64-byte buckets of two 32-byte slots
// {key dwords 0..5, info, pool offset} probed linearly bucket by bucket, so
// one probe is one cache line and a key of <= 24 bytes verifies from the
// slot alone.  info uses slot_info()'s layout; info == 0 marks an empty slot.
constexpr int VKEY_DW = 6;
constexpr uint32_t VSEED = 0x1B873593u;
LDDL_HD uint32_t vmix(uint32_t h, uint32_t d) {
  h ^= d;
  return ((h << 5) | (h >> 27)) * 0x85EBCA77u;
}
LDDL_HD uint32_t vfinal(uint32_t h, uint32_t len, uint32_t cont) {
  h ^= len * 0x9E3779B9u ^ (cont ? 0x7F4A7C15u : 0u);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return h;
}
// The scan's whole-word table (tok_tables.h build_vocab_tables): 32-B slots
// in the v4 slot layout, a key in one of two slots, at vhash & mask and at
// st_second(vhash) & mask (two-choice cuckoo placement)
LDDL_HD uint32_t st_second(uint32_t h) { return ((h >> 16) | (h << 16)) ^ 0x9E3779B9u; }
// Bucket index of a candidate piece: its first 12 bytes (three dwords, zero
// past the key), its byte length and the "##" flag -- always three mixes, so
// the scan's whole-word probe hashes a key without selecting among prefix
// mixes (no two keys of either vocab share their first 12 bytes, length and
// flag).  The WordPiece loop re-hashes a shorter candidate from the same
// three dwords (its prefix mix H3 for >= 12 bytes).
LDDL_HD uint32_t vmask_rem(uint32_t d, int rem) { return rem >= 4 ? d : rem <= 0 ? 0u : d & ((1u << (8 * rem)) - 1u); }
LDDL_HD uint32_t vhash(const uint32_t* d, uint32_t len, uint32_t cont) {
  const int l = (int)len;
  return vfinal(vmix(vmix(vmix(VSEED, vmask_rem(d[0], l)), vmask_rem(d[1], l - 4)), vmask_rem(d[2], l - 8)), len, cont);
}
// low 32 bits of the product of the low 24 bits of a and b (v_mul_u32_u24,
// full rate; a 32-bit v_mul_lo_u32 is quarter rate)
LDDL_HD uint32_t mul24(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul24(a, b);
#else
  return (a & 0xFFFFFFu) * (b & 0xFFFFFFu);
#endif
}
// Bloom key of a candidate from the mixes hq of its full dwords (first 24
// bytes), its masked partial dword (0 if none), byte length and "##" flag.
// The WordPiece scan evaluates it for every candidate length, so it avoids
// the 32-bit multiplies of vfinal; the bucket index keeps vhash.
LDDL_HD uint32_t vbkey(uint32_t hq, uint32_t tail, uint32_t len, uint32_t cont) {
  uint32_t x = hq ^ mul24(tail, 0xB5297Au) ^ mul24(len, 0x9E3779u) ^ (cont ? 0x7F4A7C15u : 0u);
  return x ^ (x >> 16);
}
LDDL_HD uint32_t vbkey_of(const uint32_t* d, uint32_t len, uint32_t cont) {
  const uint32_t l = len < 24u ? len : 24u, q = l >> 2, r = l & 3u;
  uint32_t h = VSEED;
  for (uint32_t k = 0; k < q; ++k) h = vmix(h, d[k]);
  return vbkey(h, r ? d[q] & ((1u << (8 * r)) - 1u) : 0u, len, cont);
}
// "extension" key of a prefix of 4(j+1) bytes (hq = mixes of its j+1
// dwords): in the Bloom filter iff some vocab key longer than 4(j+1) bytes
// starts with it, so the WordPiece scan never needs lengths > 4(j+1) when
// it is absent.  Tagged length (bit 23): never equal to a real key's.
constexpr uint32_t VEXT_TAG = 0x800000u;
LDDL_HD uint32_t vbkey_ext(uint32_t hq, uint32_t plen, uint32_t cont) { return vbkey(hq, 0u, VEXT_TAG | plen, cont); }
// blocked Bloom filter over the Bloom keys (BLOOM_WORDS dwords, 2 bits/key):
// word = top 13 bits, bits = two 5-bit fields below them
LDDL_HD uint32_t vbloom_word(uint32_t x) { return x >> 19; }
LDDL_HD uint32_t vbloom_bits(uint32_t x) { return (1u << ((x >> 9) & 31u)) | (1u << ((x >> 14) & 31u)); }

// ---- double-array trie of the vocab keys (tok_tables.h build_trie, tokenize_lane.h)
// Node i's child on byte c sits at base(i) + c and is valid iff its check is
// i; node 0 is the whole-word root, node 1 the "##" root (keys without the
// "##").  One 8-B entry per node, so one load per byte of a greedy
// longest-match walk:
//   x = check (bits 0-19; TRIE_EMPTY for a free slot) | id bits 0-11 << 20
//   y = base (bits 0-19) | id bits 12-15 << 20 | accept << 31
constexpr uint32_t TRIE_EMPTY = 0xFFFFFu;
LDDL_HD uint32_t trie_check(uint2 e) { return e.x & 0xFFFFFu; }
LDDL_HD uint32_t trie_base(uint2 e) { return e.y & 0xFFFFFu; }
LDDL_HD uint32_t trie_id(uint2 e) { return (e.x >> 20) | ((e.y >> 8) & 0xF000u); }
LDDL_HD bool trie_accept(uint2 e) { return (e.y >> 31) != 0u; }

// lane tokenizer byte classes (tok_tables.h lane_ctab, tokenize_lane.h): an
// ASCII word char, isolate, space, dropped control, '[', else the slow path
enum : uint32_t { LANE_CW = 1, LANE_CI = 2, LANE_CSP = 3, LANE_CDR = 4, LANE_CLB = 5, LANE_CNA = 6 };

// ---- MT19937 (CPython random) ----------------------------------------------
constexpr int MT_N = 624;
constexpr int MT_M = 397;

}  // namespace lddl
