// Kernel parameter blocks for the tokenizer (device side of lddl_tokenize).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lddl {

constexpr int WB_OVF = 384;  // per-lane overflow word buffer (bytes beyond LDS)
constexpr int TOK_WAVES = 4;        // waves per workgroup of the window kernel
constexpr int BLOOM_WORDS = 8192;   // 32 KiB blocked Bloom filter (2 bits/key)

struct TokParams {
  const uint8_t* bytes;
  const int64_t* sent_off;
  int64_t n_sent;
  int32_t max_tok;
  uint16_t* out_ids;      // dense: sentence s's ids at out_tok_off[s] (split path; the serial kernel: see below)
  int32_t* out_ntok;
  int64_t* out_tok_off;   // [n_sent + 1] exclusive scan of out_ntok
  int64_t out_cap;        // entries of out_ids
  uint8_t* sent_spec;     // optional [n_sent]: the sentence's tokens include [CLS] / [SEP]
  // unicode table
  const uint16_t* top;
  const uint32_t* pages;
  const uint4* multi;
  const uint32_t* bmp;    // [0x10000] pages[top[cp >> 8] * 256 + (cp & 255)] for cp < U+10000
  const uint32_t* xmap;   // [0x110000] the scan's fast exception entries (tokenize_split.hip XM_*)
  // vocab
  const uint4* slots;
  const uint32_t* bloom;  // [BLOOM_WORDS]
  uint32_t slot_mask;
  const uint8_t* pool;
  const uint32_t* voff;
  uint32_t maxb[2];
  uint32_t special[5];
  uint32_t unk;
  // v4 vocab table (common.h vhash): 64-B buckets of two 32-B slots + Bloom
  const uint4* vt;
  uint32_t vt_mask;  // #buckets - 1
  const uint32_t* vbloom;
  // the scan's whole-word table (two 32-B slots per key, common.h
  // st_second); null: the scan probes slot 0 of the key's vt bucket instead
  const uint4* st;
  uint32_t st_mask;
  // double-array trie of the vocab keys (common.h trie_*): the split
  // tokenizer's WordPiece walk (wpt_kernel) and the lane tokenizer
  const uint2* trie;
  uint32_t trie_base[2];  // children bases of the whole-word and "##" roots
  // scratch
  uint8_t* ovf;
  uint32_t* work_counter;
  uint64_t* dbg;  // optional phase stamps (LDDL_TOK_DEBUG=1), else null
};

int64_t tile_count(int64_t nbytes);
// tile_sent (and tile_off) of every tile, or with sup > 1 only of the tiles
// (t % seg) % sup == 0 and of n_tiles (what the split scan reads)
hipError_t launch_tile_bounds(const int64_t* sent_off, int64_t n_sent, int64_t n_tiles, int64_t* tile_sent,
                              int64_t* tile_off, hipStream_t s, int64_t seg = 0, int sup = 1);
// fb_list: *fb_count sentence ranges [fb_list[2k], fb_list[2k+1]) for the
// exact serial path (a scan window or a tile it did not model)
hipError_t launch_tokenize_fallback(const TokParams& P, const int64_t* fb_list, const int32_t* fb_count, int grid,
                                    hipStream_t s);
const void* tokenize_fallback_kernel_ptr();
// fb_list = the sentence range of every tile of [0, n_tiles), *fb_count = n_tiles
hipError_t launch_list_all_tiles(int64_t n_tiles, const int64_t* tile_sent, int64_t* fb_list, int32_t* fb_count,
                                 hipStream_t s);
// fallback ranges a segment of seg_tiles tiles can list (its scan windows)
int64_t fb_list_cap(int64_t seg_tiles);

// v5 (tokenize_split.hip): the tile scan resolves whole-word vocab hits and
// hands every other word to a WordPiece record queue; a full-occupancy
// WordPiece kernel runs the records, a count pass + scan give every
// sentence's dense offset, and an expand pass writes the dense ids.  Scratch
// per segment of tiles (SPLIT_SEG_TILES):
//   ent    u16 per byte of the segment: sentence s's entries at
//          sent_off[s] - sent_off[0] - t0 * 1 KiB + k, one per unit (k = its
//          rank in the sentence): a vocab id, SPLIT_EHOLE for an empty unit,
//          or SPLIT_EDEF | (record slot - the tile's first slot) for a word of
//          the queue (the serial path's ids of a fallback tile land here too)
//   rec    64-B record slots in chunks of SPLIT_CHUNK, chunk_fill[c] used;
//          a tile's slots contiguous, in unit order
//   smeta  per sentence: #entries | first slot relative to the tile's << 16,
//          the tile's first slot
// 8 GiB of input per segment: ~100 GB of scratch (entries 2 B/byte, record
// slots and WordPiece outputs 64 B per 14 B each); fewer kernel boundaries
// and launch tails than 4 GiB segments (3 launches per kernel for the 21.4 GB
// bench step instead of 5: 112.6 -> 110.9 ms, profiles/r6/seg/; earlier 4 vs
// 1 GiB: 246.7 vs 250.8 ms).  The masked bench at 20 GB of corpus still leaves
// ~50 GB of the 309 GB free (hbm_free_gb in the bench legs).
constexpr int64_t SPLIT_SEG_TILES = int64_t(1) << 23;
constexpr uint32_t SPLIT_CHUNK = 1024;                 // record slots per allocation chunk (64 KiB)
constexpr uint32_t SPLIT_EDEF = 0xF000u;               // entry >= EDEF: a queued word
constexpr uint16_t SPLIT_NENT_FB = 0xFFFFu;            // nent of a sentence of a fallback tile
constexpr uint16_t SPLIT_EHOLE = 0xFFFFu;              // entry of an empty unit (no token)

struct SplitParams {
  int64_t seg_tiles;       // tiles per segment (SPLIT_SEG_TILES; tests force small ones)
  int64_t t0, t1;          // the segment's tiles
  const int64_t* tile_sent;
  const int64_t* tile_off;  // sent_off[tile_sent[t]] (the scan stages a tile's bounds in one round trip)
  uint16_t* ent;
  uint4* rec;              // 4 uint4 per slot
  uint4* pcs;              // WordPiece pieces 4.. per slot (64 B per slot; the extension slot continues it)
  uint4* pch;              // WordPiece head per slot: {#pieces, pieces 0-1, pieces 2-3, 0}: dense 16 B, what
                           // expand reads for nearly every record (one 16-B line share instead of a 64-B stride)
  uint32_t* chunk_fill;
  uint32_t* chunk_ctr;     // [0] chunks handed out by the scan, [1] by wp_kernel, [2] super-tiles claimed by the scan
  uint32_t n_chunks;
  uint2* smeta;            // per sentence: #entries | first slot - the tile's << 16, the tile's first slot
  uint16_t* snslot;        // per sentence: its record slots (count_kernel sums their piece counts)
  uint8_t* cnt8;           // per record slot: pieces of the word (0 for an extension slot)
  int64_t* scan_bsum;      // scan_blocks(seg_sent_cap) + 1
  int64_t seg_sent_cap;    // bound on the sentences of a segment (the count scan's grid)
  int64_t* fb_list;        // sentence ranges for the serial path (pairs, launch_tokenize_fallback)
  int32_t* fb_count;       // ranges listed in this segment
  uint32_t* n_fallback;    // tiles listed over the call (lddl_tokenize_stats)
  unsigned long long* n_rec;  // optional: records run by wp_kernel (summed over the call)
};
// optional per-kernel timing of a call: event pairs recorded around every
// launch (scan / wp / expand per segment)
struct SplitTiming {
  hipEvent_t ev[3][2][64];
  int n[3];
};
hipError_t launch_tokenize_split(const TokParams& P, int64_t nbytes, int64_t* tile_sent, SplitParams S, int n_cu,
                                 int fb_grid, hipStream_t s, SplitTiming* tm = nullptr);
// every tile through the exact serial path, same dense output (tables the
// split tokenizer does not model, LDDL_TOKENIZE_ALGO=0)
hipError_t launch_tokenize_serial_dense(const TokParams& P, int64_t nbytes, int64_t* tile_sent, SplitParams S,
                                        int n_cu, int fb_grid, hipStream_t s);
// record slots for a segment: 1 per 14 input bytes + a partly used chunk per
// scanning wave of the scan's real grid on n_cu CUs
int64_t split_seg_slots(int64_t seg_tiles, int n_cu);

// lane tokenizer (tokenize_lane.hip, tokenize_lane.h)
namespace tok6 {
struct LaneParams {
  const uint2* trie;
  uint32_t rbase[2];      // children bases of the two roots
  uint16_t* stage;        // ids at (sentence byte offset - segb)
  int64_t segb;           // absolute byte offset of staging index 0 (the host passes t0 << 10;
                          // the kernels add sent_off[0])
  int64_t bytes_end;      // absolute end of the corpus (set on the device; ring loads start below it)
  const int64_t* tile_sent;
  const int64_t* tile_off;
  int64_t t0, t1;         // the segment's tiles
  uint32_t* ctr;          // [0] tile batches handed out
  int64_t* fb_list;       // sentence-range pairs (SplitParams::fb_list)
  int32_t* fb_count;
  uint32_t* n_fallback;
  uint64_t* stats;        // optional: [0] iterations x 64, [1] lane-iterations busy, [2] slow passes
};
}  // namespace tok6
hipError_t launch_tokenize_lane(const TokParams& P, int64_t nbytes, int64_t* tile_sent, SplitParams S,
                                tok6::LaneParams Q, const uint16_t* d_ctab, int n_cu, int fb_grid, hipStream_t s,
                                SplitTiming* tm);

}  // namespace lddl
