#!/bin/bash
# Build the library of a git revision (default HEAD) into ab/lib_<name>.so for
# A/B runs against the working tree (tools/r2_ab.sh LIBS=...).
#   tools/ab_head.sh [REV] [NAME]
set -e
REV=${1:-HEAD}; NAME=${2:-head}
ROOT=$(cd $(dirname $0)/.. && pwd)
WT=$(mktemp -d /tmp/lddl_wt.XXXX)
git -C $ROOT worktree add -q --detach $WT $REV
mkdir -p $ROOT/ab
(cd $WT && python -c "
import sys; sys.path.insert(0, '.')
from lddl_amd import build
print(build.build_hip(force=True, lib='$ROOT/ab/lib_$NAME.so'))") > /tmp/ab_$NAME.log 2>&1 || { tail /tmp/ab_$NAME.log; git -C $ROOT worktree remove --force $WT; exit 1; }
git -C $ROOT worktree remove --force $WT
ls -la $ROOT/ab/lib_$NAME.so
