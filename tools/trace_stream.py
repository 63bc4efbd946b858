"""Timeline of the streaming (host-fed) bench from a rocprofv3 kernel trace:
per fingerprint pass its duration and the time it waited behind the previous
SHA-256 slice; SHA-256 slice durations.  usage: trace_stream.py <kernel_trace.csv>"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    fp = [(a, b) for a, b, n in ev if "fp_kernel" in n]
    sha = [(a, b) for a, b, n in ev if "sha_slice" in n]
    t0 = ev[0][0]
    print(f"kernels {len(ev)}  fp {len(fp)}  sha slices {len(sha)}")
    if fp:
        d = sorted((b - a) / 1e6 for a, b in fp)
        print(f"fp ms: min {d[0]:.3f} median {d[len(d) // 2]:.3f} max {d[-1]:.3f} total {sum(d):.1f}")
        gaps = sorted((fp[i + 1][0] - fp[i][1]) / 1e6 for i in range(len(fp) - 1))
        if gaps:
            print(f"gap between fp passes ms: median {gaps[len(gaps) // 2]:.3f} max {gaps[-1]:.3f}")
    if sha:
        d = sorted((b - a) / 1e6 for a, b in sha)
        print(f"sha slice ms: min {d[0]:.3f} median {d[len(d) // 2]:.3f} max {d[-1]:.3f} total {sum(d):.1f}")
    # first 40 events of the steady state
    mid = len(ev) // 2
    for a, b, n in ev[mid:mid + 40]:
        print(f"{(a - t0) / 1e6:10.3f} {(b - a) / 1e6:8.3f}  {n.split('(')[0][-40:]}")


if __name__ == "__main__":
    main()
