#!/bin/bash
# The SSA event loop's ceiling on this chip (scripts/loop_ceiling.hip): lane-events/s of the library's own event loop
# with every lane busy, per BASELINE config, eight waves per SIMD (8,192 one-wave blocks, one round of the grid), then a
# rocprofv3 PMC pass of the same dispatches (wave64 VALU instructions per second, VALU busy).
# scripts/loop_ceiling_parse.py writes gpurun_out/ceiling/loop_ceiling.json (copied to profiles/ for bench.py).
# The binary (scripts/bin/loop_ceiling) is built by __graft_entry__.build() in the build container.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ceiling
mkdir -p $OUT
B=scripts/bin/loop_ceiling
[ -x $B ] || { echo "$B is not built"; exit 1; }
timeout -k 10 180 $B "" 8192 0 > $OUT/natural.jsonl || exit $?
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE \
  --kernel-include-regex loop_ceiling -d $OUT/pmc -o run --output-format csv -- $B "" 8192 0 > $OUT/pmc.log 2>&1 || exit $?
python3 scripts/loop_ceiling_parse.py $OUT > $OUT/loop_ceiling.json || exit $?
cat $OUT/loop_ceiling.json
