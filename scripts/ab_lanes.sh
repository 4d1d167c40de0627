#!/bin/bash
# A/B of whole one-to-few-chain filters (scripts/lanes_sweep.py) between the tree in $AB_DIR (default ab_old: a worktree
# of another commit, built in place) and this tree, alternating on one box.  Arguments go to lanes_sweep.py.  B_LIB: a
# library of this tree other than lib/libepipf.so for side B (EPIPF_LIBRARY), e.g. a variant built with another OUT.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab_lanes}
mkdir -p $OUT
ROOT=$(pwd)
for i in ${ROUNDS:-1 2}; do
  for side in A B; do
    dir=$ROOT; [ $side = A ] && dir=$ROOT/${AB_DIR:-ab_old}
    lib=; [ $side = B ] && [ -n "${B_LIB:-}" ] && lib=$ROOT/$B_LIB
    (cd $dir && env ${lib:+EPIPF_LIBRARY=$lib} timeout -k 10 ${T_LIMIT:-240} python scripts/lanes_sweep.py --out $ROOT/$OUT/$side$i.jsonl "$@") \
      > $OUT/$side$i.log 2>&1 || { echo "STOP $side$i rc=$?"; tail -5 $OUT/$side$i.log; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import json, sys, glob, collections
d = collections.defaultdict(list)
for p in sorted(glob.glob(sys.argv[1] + "/*.jsonl")):
    side = p.split("/")[-1][0]
    for line in open(p):
        r = json.loads(line)
        d[(r["cfg"], r["chains"], r["lanes"], side)].append(r["particle_steps_per_s"])
keys = sorted({k[:3] for k in d})
for k in keys:
    a, b = d.get(k + ("A",), []), d.get(k + ("B",), [])
    if a and b:
        ma, mb = max(a), max(b)
        print(f"cfg {k[0]} chains {k[1]} lanes {k[2]}: A {ma:.4e} B {mb:.4e} B/A {mb / ma:.3f}")
PY
