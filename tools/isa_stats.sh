#!/bin/bash
# Register / spill / occupancy figures of every kernel in a HIP source
#   tools/isa_stats.sh lddl_amd/csrc/tokenize_split.hip [extra hipcc flags]
SRC=$(realpath $1); shift
D=$(mktemp -d /tmp/isa.XXXX)
(cd $D && hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c --save-temps -o $D/x.o $SRC "$@" 2>/dev/null)
S=$(ls $D/*gfx950.s)
python3 - "$S" <<'PY'
import re, sys
s = open(sys.argv[1]).read()
for m in re.finditer(r'\.name:\s+(\S+)\n(.*?)(?=\n  - \.|\n\.end_amdgpu_metadata)', s, re.S):
  name, body = m.group(1), m.group(2)
  g = lambda k: (re.search(r'\.%s:\s+(\d+)' % k, body) or [None, '?'])[1]
  print('%-60s vgpr %3s agpr %3s sgpr %3s vspill %3s sspill %3s scratch %4s lds %6s' % (
      name[:60], g('vgpr_count'), g('agpr_count'), g('sgpr_count'), g('vgpr_spill_count'), g('sgpr_spill_count'),
      g('private_segment_fixed_size'), g('group_segment_fixed_size')))
PY
rm -rf $D
