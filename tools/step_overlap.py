"""Overlap of one training step in a rocprofv3 --kernel-trace database: the kernels between
the last two optimizer launches (yxh sgd_ema_step), their sum of durations, the busy time
(union of kernel intervals), the time two or more kernels ran at once, and the split over
hardware queues.  Usage: python tools/step_overlap.py <results.db>"""
import sqlite3
import sys
from collections import Counter


def main(path: str) -> None:
    c = sqlite3.connect(path)
    rows = c.execute("select name, queue_id, start, end from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if "sgd" in r[0].lower()]
    if len(idx) < 2:
        sys.exit("fewer than two optimizer launches in the trace")
    step = rows[idx[-2] + 1:idx[-1] + 1]
    t0, t1 = step[0][2], max(r[3] for r in step)
    ev = sorted([(r[2], 1) for r in step] + [(r[3], -1) for r in step])
    busy = over = 0
    cur, last = 0, t0
    for t, d in ev:
        if cur > 0:
            busy += t - last
        if cur > 1:
            over += t - last
        cur += d
        last = t
    print(f"kernels {len(step)}  span {(t1 - t0) / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  "
          f"concurrent {over / 1e6:.3f} ms  sum of durations {sum(r[3] - r[2] for r in step) / 1e6:.3f} ms")
    for q, n in sorted(Counter(r[1] for r in step).items()):
        wg = sum(1 for r in step if r[1] == q and "wgrad" in r[0])
        ms = sum(r[3] - r[2] for r in step if r[1] == q) / 1e6
        print(f"  queue {q}: {n} kernels ({wg} weight-gradient), {ms:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
