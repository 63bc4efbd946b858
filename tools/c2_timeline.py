"""Timeline of a C2 bench run from a rocprofv3 kernel trace (fp_kernel and
sha_slice_kernel dispatches): every pass and slice in start order with its
start time (ms, from the first dispatch), duration and the gaps in which no
hot kernel ran, then per-kernel busy totals.  usage: c2_timeline.py <kernel_trace.csv>"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].split("(")[0].replace("void ", "").replace("vsgpu::", ""))
                for r in rows)
    ev = [e for e in ev if "fp_kernel" in e[2] or "sha_slice" in e[2]]
    if not ev:
        print("no hot kernels")
        return
    t0 = ev[0][0]
    end = t0
    busy = {}
    idle = 0
    for a, b, n in ev:
        gap = (a - end) / 1e6
        if gap > 0:
            idle += gap
        mark = f"   <idle {gap:.2f} ms>" if gap > 0.5 else ""
        print(f"{(a - t0) / 1e6:10.2f} {(b - a) / 1e6:9.2f}  {n[-28:]}{mark}")
        busy[n] = busy.get(n, 0.0) + (b - a) / 1e6
        end = max(end, b)
    print(f"span {(end - t0) / 1e6:.1f} ms, no hot kernel running {idle:.1f} ms")
    for n, v in busy.items():
        print(f"  {n}: {v:.1f} ms busy")


if __name__ == "__main__":
    main()
