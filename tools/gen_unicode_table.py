#!/usr/bin/env python3
"""Generate the per-code-point BertNormalizer / BertPreTokenizer table.

Run HERE (the build container), never on the GPU box.  Source of truth: the
HF ``tokenizers`` wheel (0.22.2) that ``transformers.BertTokenizerFast`` wraps
in the reference (``lddl/dask/bert/pretrain.py:584-587``, ``:79-80``).  The
reference pins ``transformers==4.16.2`` (``setup.py:55``) but not the tokenizers
version; 0.22.2 is the version pinned here (DESIGN.md "Oracle").

For every code point c (surrogates excluded) we record

  * ``normalize_str(c)``  -- BertNormalizer(clean_text, handle_chinese_chars,
    strip_accents=lowercase, lowercase) applied to the single char,
  * the BertPreTokenizer class of every output char (space / isolate / other),
  * the canonical-reordering rank of every surviving char (NFD orders runs of
    ccc>0 chars; only 80 survivors have ccc>0 in the crate's Unicode tables),
  * for chars normalised away: whether they are transparent to a ccc run
    (removed Mn with ccc>0, removed controls) or delimit it (removed Mn, ccc=0).

Everything is measured by probing tokenizers with crafted strings; the result
is checked against whole-string normalisation on fuzz strings before writing.

Output: lddl_amd/data/unicode_table.bin (format in lddl_amd/csrc/unicode_table.h)
        tests/golden/normalize_fuzz.json
"""
import collections
import json
import os
import random
import struct
import sys

import numpy as np
import transformers

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VOCAB = '/root/reference/lddl/dask/bert/vocab'

KIND_IDENT, KIND_MAP, KIND_DROP_T, KIND_DROP_D, KIND_MULTI = 0, 1, 2, 3, 4
CLS_OTHER, CLS_SPACE, CLS_ISOLATE = 0, 1, 2

P = '\U0001D16D'  # surviving mark, ccc 226
S = '\U0001D165'  # surviving mark, ccc 216


def main():
    tok = transformers.BertTokenizerFast(VOCAB)
    norm = tok.backend_tokenizer.normalizer
    pre = tok.backend_tokenizer.pre_tokenizer
    N = norm.normalize_str

    cps = [cp for cp in range(0x110000) if not (0xD800 <= cp < 0xE000)]
    outs = {cp: N(chr(cp)) for cp in cps}

    cls = {}
    for cp in cps:
        r = pre.pre_tokenize_str('a' + chr(cp) + 'b')
        cls[cp] = {1: CLS_OTHER, 2: CLS_SPACE, 3: CLS_ISOLATE}[len(r)]
    assert all(cls[ord(ch)] != CLS_SPACE or ch == ' ' for o in outs.values() for ch in o)

    # --- canonical reordering participants (chars that survive with ccc>0) ---
    part = set()
    for cp, o in outs.items():
        if not o:
            continue
        c = chr(cp)
        if N(P + c) != outs[ord(P)] + o or N(c + P) != o + outs[ord(P)]:
            part.add(cp)
    part.add(ord(P))
    # every participant is identity-mapped (checked)
    assert all(outs[cp] == chr(cp) for cp in part)
    # rank = number of participants that sort strictly before it
    pl = sorted(part)
    less = collections.defaultdict(int)
    for x in pl:
        for y in pl:
            if x != y and N(chr(x) + chr(y)) != chr(x) + chr(y):
                less[x] += 1  # y moved before x  => ccc(y) < ccc(x)
    levels = sorted(set(less[x] for x in pl))
    rank = {x: levels.index(less[x]) + 1 for x in pl}
    assert max(rank.values()) <= 7

    drop_kind = {}
    for cp, o in outs.items():
        if o:
            continue
        r = N(P + chr(cp) + S)
        if r == S + P:
            drop_kind[cp] = KIND_DROP_T
        elif r == P + S:
            drop_kind[cp] = KIND_DROP_D
        else:
            raise AssertionError(hex(cp))

    def item(ch):
        c = ord(ch)
        return c | (rank.get(c, 0) << 21) | (cls[c] << 24)

    multi = []  # list of tuples of items
    multi_idx = {}
    entries = np.zeros(0x110000, dtype=np.uint32)
    for cp in range(0x110000):
        if 0xD800 <= cp < 0xE000:
            entries[cp] = KIND_DROP_T << 26
            continue
        o = outs[cp]
        if not o:
            e = drop_kind[cp] << 26
        elif len(o) == 3 and o[0] == ' ' and o[2] == ' ':
            # CJK padding: the char becomes its own word == isolate class
            inner = ord(o[1])
            assert rank.get(inner, 0) == 0
            if inner == cp:
                e = (KIND_IDENT << 26) | (CLS_ISOLATE << 24)
            else:
                e = (KIND_MAP << 26) | (CLS_ISOLATE << 24) | inner
        elif len(o) == 1:
            it = item(o)
            if ord(o) == cp:
                e = (KIND_IDENT << 26) | (it & ~0x1FFFFF)
            else:
                e = (KIND_MAP << 26) | it
        else:
            key = tuple(item(ch) for ch in o)
            if key not in multi_idx:
                multi_idx[key] = len(multi)
                multi.append(key)
            e = (KIND_MULTI << 26) | multi_idx[key]
        entries[cp] = e

    # --- two-level table: unique 256-entry pages ---
    pages = []
    page_idx = {}
    top = np.zeros(0x1100, dtype=np.uint16)
    for p in range(0x1100):
        blk = entries[p * 256:(p + 1) * 256].tobytes()
        if blk not in page_idx:
            page_idx[blk] = len(pages)
            pages.append(blk)
        top[p] = page_idx[blk]
    mult = np.zeros((len(multi), 4), dtype=np.uint32)
    for i, key in enumerate(multi):
        mult[i, 0] = len(key)
        mult[i, 1:1 + len(key)] = key

    # --- self check: decode table == per-char outputs ---
    def decode(cp):
        e = int(entries[cp])
        kind = e >> 26
        if kind == KIND_IDENT:
            return chr(cp)
        if kind == KIND_MAP:
            return chr(e & 0x1FFFFF)
        if kind in (KIND_DROP_T, KIND_DROP_D):
            return ''
        k = mult[e & 0x1FFFFF]
        return ''.join(chr(int(k[1 + j]) & 0x1FFFFF) for j in range(int(k[0])))

    for cp in cps:
        o = outs[cp]
        if len(o) == 3 and o[0] == ' ' and o[2] == ' ':
            o = o[1]
        assert decode(cp) == o, hex(cp)

    out_path = os.path.join(ROOT, 'lddl_amd', 'data', 'unicode_table.bin')
    with open(out_path, 'wb') as f:
        f.write(struct.pack('<8sIII', b'LDDLUNI1', len(pages), len(multi), 0))
        f.write(top.tobytes())
        for blk in pages:
            f.write(blk)
        f.write(mult.tobytes())
    print('pages', len(pages), 'multi', len(multi), 'participants', len(part),
          'bytes', os.path.getsize(out_path))

    # --- fuzz fixture: normalise + pre-tokenise whole strings (reordering cases) ---
    rng = random.Random(20261015)
    pool = (list(part) + [ord(c) for c in 'aAbZ09 .,-_#[]'] +
            [0x1D15E, 0x1D160, 0x1D1BD, 0x300, 0x301, 0x327, 0x34F, 0x941,
             0x0130, 0x03A3, 0x00E9, 0xAC00, 0xD55C, 0x4E2D, 0xF900, 0x200B,
             0xFEFF, 0x0085, 0x00A0, 0x3000, 0x2028, 0x0000, 0xFFFD, 0x0007])
    pool += rng.sample(cps, 200)
    pool += [cp for cp, k in drop_kind.items() if k == KIND_DROP_D][:40]
    cases = []
    for _ in range(4000):
        n = rng.randint(1, 12)
        s = ''.join(chr(rng.choice(pool)) for _ in range(n))
        cases.append([s, [w for w, _ in pre.pre_tokenize_str(N(s))]])
    with open(os.path.join(ROOT, 'tests', 'golden', 'normalize_fuzz.json'),
              'w', encoding='utf-8') as f:
        json.dump({'generator': 'tools/gen_unicode_table.py',
                   'tokenizers': __import__('tokenizers').__version__,
                   'cases': cases}, f, ensure_ascii=True)


if __name__ == '__main__':
    sys.exit(main())
