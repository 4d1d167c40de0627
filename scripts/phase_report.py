"""Summarise the per-wave phase cycles printed by the phase-timing build of the lane-group step kernel (make phase:
lib/libepipf_phase.so, s_memtime at the phase fences of group_propagate; diagnostic only).

    python scripts/phase_report.py log..."""
import collections
import re
import sys

pat = re.compile(r"PH p=(\d+) b=(\d+) w=(\d+) ch=(\d+) pre=(\d+) ssa=(\d+) bar=(\d+) post=(\d+) draws=(\d+) "
                 r"decide=(\d+) ball=(\d+) tau=(\d+) clock=(\d+) nev=(-?\d+)")
for f in sys.argv[1:]:
    steps = collections.defaultdict(list)
    for line in open(f):
        m = pat.search(line)
        if m:
            v = list(map(int, m.groups()))
            steps[v[0]].append(v)
    tot = collections.Counter()
    crit = collections.Counter()
    n_ch = crit_ch = 0
    for p, rows in sorted(steps.items()):
        slow = max(rows, key=lambda r: r[5])
        crit_ch += slow[3]
        for k, i in (("pre", 4), ("ssa", 5), ("bar", 6), ("post", 7), ("draws", 8), ("decide", 9), ("ball", 10),
                     ("tau", 11), ("clock", 12)):
            crit[k] += slow[i]
            tot[k] += sum(r[i] for r in rows)
        n_ch += sum(r[3] for r in rows)
    print(f"== {f}: {len(steps)} steps")
    print("critical waves (slowest SSA per step), cycles per chunk:",
          {k: round(crit[k] / max(crit_ch, 1), 1) for k in ("ssa", "draws", "decide", "ball", "tau", "clock")},
          "chunks", crit_ch, "ssa cycles", crit["ssa"], "pre", crit["pre"], "post", crit["post"])
    print("all waves, cycles per chunk:",
          {k: round(tot[k] / max(n_ch, 1), 1) for k in ("ssa", "draws", "decide", "ball", "tau", "clock")})
