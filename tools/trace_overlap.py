"""Per-kernel launch durations of a rocprofv3 kernel trace, split into launches that ran
alone and launches that overlapped another kernel (another HIP stream's, on another hardware
queue: the tracer does not serialise queues). An overlapped launch's span includes the time
its workgroups waited for CUs the other kernel held, so its mean says little about the
kernel itself. usage: python tools/trace_overlap.py run_kernel_trace.csv [name-substring ...]"""
import csv
import statistics
import sys


def main(path, names):
    rows = list(csv.DictReader(open(path)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    starts = [x[0] for x in iv]
    import bisect
    by = {}
    for k, (s, e, n) in enumerate(iv):
        short = n.split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
        if names and not any(x in n for x in names):
            continue
        # any other launch with start < e and end > s (scan the launches that started before e)
        hi = bisect.bisect_left(starts, e)
        ov = any(j != k and iv[j][1] > s for j in range(max(0, k - 2000), hi))
        by.setdefault(short, ([], []))[1 if ov else 0].append((e - s) / 1000.0)
    print("%-24s %6s %9s %9s | %6s %9s %9s %9s" % ("kernel", "alone", "median", "mean", "overl", "median", "mean", "max"))
    for short, (a, o) in sorted(by.items(), key=lambda kv: -sum(kv[1][0] + kv[1][1])):
        f = lambda v, g: "%9.1f" % g(v) if v else "%9s" % "-"
        print("%-24s %6d %s %s | %6d %s %s %s" % (short[:24], len(a), f(a, statistics.median), f(a, statistics.mean),
                                                 len(o), f(o, statistics.median), f(o, statistics.mean), f(o, max)))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
