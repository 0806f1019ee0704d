"""Critical path of the forward sync-free sweep from per-item stamps
(IPO_SF_STAMPS_FILE written by a -DIPO_SF_STAMPS build; developer tool).
usage: sf_critical.py <items.txt>"""
import sys
from collections import defaultdict


def main():
    items = []
    for line in open(sys.argv[1]):
        s, c, lv, par, *t = map(int, line.split())
        ne = t[6] if len(t) > 6 else 0
        extra = t[7:9] if len(t) > 8 else [0, 0]
        items.append(dict(s=s, c=c, lv=lv, par=par, t=t[:6], ne=ne, x=extra))
    bysup, children = defaultdict(list), defaultdict(list)
    for it in items:
        bysup[it["s"]].append(it)
        if it["c"] != -2 and it["par"] >= 0:
            children[it["par"]].append(it)

    def deps(it):
        return children.get(it["s"], []) if it["c"] < 0 else [x for x in bysup[it["s"]] if x["c"] == -2]
    cur = max(items, key=lambda x: x["t"][4])
    path = []
    while True:
        path.append(cur)
        d = deps(cur)
        if not d:
            break
        cur = max(d, key=lambda x: x["t"][3])
    path.reverse()
    tot = defaultdict(float)
    for a, b in zip([None] + path, path):
        if a is not None:
            tot["handoff"] += b["t"][1] - a["t"][3]
        tot["diag" if b["c"] < 0 else "chunk wait->zl"] += b["t"][2] - b["t"][1]
        tot["rest"] += b["t"][3] - b["t"][2]
    print(f"critical path: {len(path)} items, span {path[-1]['t'][4] / 100:.1f} us")
    for k, v in tot.items():
        print(f"  {k:16s} {v / 100:8.1f} us")
    for it in path[-10:]:
        t = it["t"]
        g = (t[5] - t[1]) / 100 if it["c"] < 0 and len(t) > 5 else 0.0
        print("  level", it["lv"], "sup", it["s"], "code", it["c"], "gather", g, "diag", (t[2] - t[1]) / 100,
              "rest", (t[3] - t[2]) / 100, "list entries", it["ne"],
              "ptr loaded", (it["x"][0] - t[1]) / 100, "values summed", (it["x"][1] - t[1]) / 100)


if __name__ == "__main__":
    main()
