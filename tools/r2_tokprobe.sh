set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2_tokprobe; mkdir -p $OUT
timeout -k 10 300 python tools/tok_check.py 256 4:4 > $OUT/check.log 2>&1 || exit $?
LDDL_TOK_ABLATE=1 timeout -k 10 300 python tools/tok_check.py 256 4:4 > $OUT/ablate1.log 2>&1 || exit $?
LDDL_TOK_DEBUG=1 timeout -k 10 300 python tools/tok_check.py 256 4:0 > $OUT/dbg.log 2>&1 || exit $?
grep -h "variant\|dbg" $OUT/*.log | tail -20
