"""Timeline of the last bench round from a rocprofv3 kernel trace (csv):
every kernel of the last `--span` ms with its start offset, duration and
queue, then per queue the busy time and the idle gaps.  Measurement aid only.

usage: python scripts/exp/timeline.py run_kernel_trace.csv [--span 30] [--top 60]
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--span", type=float, default=30.0, help="ms before the last kernel's end")
    ap.add_argument("--top", type=int, default=80)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?"),
                         r.get("Stream_Id", "?"), r["Kernel_Name"][:70]))
    rows.sort()
    t_end = max(e for _, e, *_ in rows)
    t0 = t_end - a.span * 1e6
    sel = [r for r in rows if r[0] >= t0]
    base = sel[0][0]
    print(f"{len(sel)} kernels in the last {a.span} ms")
    for s, e, q, st, n in sel[: a.top]:
        print(f"{(s - base) / 1e6:9.3f} {(e - s) / 1e3:9.1f}us q{q} s{st} {n}")
    byq = defaultdict(list)
    for s, e, q, st, n in sel:
        byq[q].append((s, e))
    for q, iv in byq.items():
        iv.sort()
        busy, gaps, cur_s, cur_e = 0, [], iv[0][0], iv[0][1]
        for s, e in iv[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                gaps.append((cur_e - base, s - cur_e))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        big = sorted(gaps, key=lambda g: -g[1])[:8]
        print(f"queue {q}: {len(iv)} kernels, busy {busy / 1e6:.3f} ms, "
              f"gaps {sum(g for _, g in gaps) / 1e6:.3f} ms; largest: " +
              ", ".join(f"{g / 1e3:.0f}us@{s / 1e6:.2f}" for s, g in big))


if __name__ == "__main__":
    main()
