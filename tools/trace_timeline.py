"""Timeline of a rocprofv3 kernel + memory-copy trace (csv output): every kernel and copy in
order, relative to the first event of the last `--window` milliseconds, with its duration and
queue / stream.  Usage: trace_timeline.py <trace dir> [--window MS] [--min-us US]"""
import argparse
import csv
import glob
import os


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--window", type=float, default=20.0)
    ap.add_argument("--min-us", type=float, default=0.0)
    a = ap.parse_args()
    ev = []
    for r in rows(a.dir, "*kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:60],
                   r.get("Queue_Id", "?"), r.get("Stream_Id", "?")))
    for r in rows(a.dir, "*memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", r.get("Direction", "copy") + " " +
                   r.get("Bytes", r.get("Size", "?")), r.get("Queue_Id", "-"), r.get("Stream_Id", "-")))
    ev.sort()
    if not ev:
        print("no events")
        return
    end = max(e[1] for e in ev)
    t0 = None
    for s, e, k, name, q, st in ev:
        if s < end - a.window * 1e6:
            continue
        if t0 is None:
            t0 = s
        if (e - s) / 1e3 < a.min_us:
            continue
        print(f"{(s - t0) / 1e6:9.3f} .. {(e - t0) / 1e6:9.3f} ms  {(e - s) / 1e3:9.1f} us  {k} q{q} s{st}  {name}")


if __name__ == "__main__":
    main()
