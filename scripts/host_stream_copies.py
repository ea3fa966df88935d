#!/usr/bin/env python3
"""Summarise one host-stream process's copies from its rocpd database: per direction, the queues/streams the copies
ran on, bytes, busy time and rate, and how long both directions were in flight at once.  Prints one JSON line."""
import json
import sqlite3
import sys


def main(db, result_json=None):
    c = sqlite3.connect(db)
    rows = c.execute("select start, end, size, src_agent_type, dst_agent_type, queue_name, stream_name, name "
                     "from memory_copies").fetchall()
    out = {"db": db}
    if result_json:
        try:
            r = json.loads(open(result_json).read().strip().splitlines()[-1])
            out["value"] = r["pinned"]["value"]
            out["step_ms"] = r["pinned"]["step_ms"]
        except Exception:
            pass
    dirs = {}
    for s, e, size, sa, da, q, st, name in rows:
        d = f"{sa}->{da}"
        x = dirs.setdefault(d, {"copies": 0, "bytes": 0, "busy_ns": 0, "queues": {}, "names": {}})
        x["copies"] += 1
        x["bytes"] += size
        x["busy_ns"] += e - s
        key = f"{q}/{st}"
        x["queues"][key] = x["queues"].get(key, 0) + 1
        x["names"][name] = x["names"].get(name, 0) + 1
    for d, x in dirs.items():
        x["GBps_while_busy"] = round(x["bytes"] / max(1, x["busy_ns"]), 2)
    # overlap of the big CPU->GPU and GPU->CPU copies (>= 1 MiB)
    h2d = sorted((s, e) for s, e, size, sa, da, *_ in rows if sa == "CPU" and da == "GPU" and size >= 1 << 20)
    d2h = sorted((s, e) for s, e, size, sa, da, *_ in rows if sa == "GPU" and da == "CPU" and size >= 1 << 20)

    def union(iv):
        tot, cur = 0, None
        for s, e in iv:
            if cur is None or s > cur[1]:
                if cur:
                    tot += cur[1] - cur[0]
                cur = [s, e]
            else:
                cur[1] = max(cur[1], e)
        return tot + (cur[1] - cur[0] if cur else 0), iv

    def inter(a, b):
        i = j = tot = 0
        while i < len(a) and j < len(b):
            s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
            if s < e:
                tot += e - s
            if a[i][1] < b[j][1]:
                i += 1
            else:
                j += 1
        return tot

    def merged(iv):
        m = []
        for s, e in iv:
            if m and s <= m[-1][1]:
                m[-1][1] = max(m[-1][1], e)
            else:
                m.append([s, e])
        return m

    mh, md = merged(h2d), merged(d2h)
    out["h2d_busy_ms"] = round(sum(e - s for s, e in mh) / 1e6, 2)
    out["d2h_busy_ms"] = round(sum(e - s for s, e in md) / 1e6, 2)
    out["both_busy_ms"] = round(inter(mh, md) / 1e6, 2)
    out["directions"] = dirs
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
