"""Diagnostic: GPU timeline of the last C4 update from a rocprofv3 kernel trace (tools/gpu_r04s.sh).

    python tools/c4_timeline.py gpurun_out/r04/c4kt/.../kt_kernel_trace.csv [window_ms]

Takes the last `window_ms` (default: one update, 760 ms) of the trace and reports: the union of kernel
intervals (GPU busy), idle time, the busy time per stream (Queue_Id) and the top kernels by total duration,
each with the share of its time spent while another queue's kernel overlapped it.
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    win = float(sys.argv[2]) if len(sys.argv) > 2 else 760.0
    rows = [r for r in csv.DictReader(open(path))]
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70], r.get("Queue_Id", "?"))
          for r in rows]
    ev.sort()
    t_end = max(e for _, e, _, _ in ev)
    t0 = t_end - win * 1e6
    ev = [x for x in ev if x[0] >= t0]
    # union of intervals
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in ev:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = ev[-1][1] - ev[0][0]
    print("window %.1f ms: %d kernels, span %.1f ms, GPU busy (union) %.1f ms, idle %.1f ms"
          % (win, len(ev), span / 1e6, busy / 1e6, (span - busy) / 1e6))
    per_q = collections.defaultdict(float)
    for s, e, _, q in ev:
        per_q[q] += e - s
    for q, t in sorted(per_q.items()):
        print("  queue %s: kernel time %.1f ms" % (q, t / 1e6))
    tot = collections.defaultdict(lambda: [0, 0.0])
    for s, e, n, _ in ev:
        tot[n][0] += 1
        tot[n][1] += e - s
    print("top kernels:")
    for n, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:25]:
        print("  %-70s %6d calls %9.2f ms %8.1f us" % (n, c, t / 1e6, t / c / 1e3))
    # gaps larger than 20 us on the busiest queue
    q0 = max(per_q, key=per_q.get)
    qe = [(s, e) for s, e, _, q in ev if q == q0]
    gaps = [qe[i + 1][0] - qe[i][1] for i in range(len(qe) - 1)]
    big = [g for g in gaps if g > 20000]
    print("queue %s: %d gaps > 20 us totalling %.1f ms; all gaps %.1f ms" % (q0, len(big), sum(big) / 1e6,
                                                                            sum(g for g in gaps if g > 0) / 1e6))


if __name__ == "__main__":
    main()
