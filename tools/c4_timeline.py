"""Timeline of the last bench step from a rocprofv3 run with --kernel-trace
--hip-runtime-trace --memory-copy-trace: GPU activities (kernels, copies) and
the HIP API calls longer than 0.2 ms, in time order, with the idle gaps of the
GPU between activities.  usage: c4_timeline.py <rocprof output dir>"""
import csv
import glob
import os
import sys


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        out.extend(csv.DictReader(open(f)))
    return out


def main():
    d = sys.argv[1]
    ev = []
    for r in rows(d, "*kernel_trace.csv"):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K",
                   name.split("(")[0].replace("void ", "")[-48:]))
    for r in rows(d, "*memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C",
                   f"{r.get('Direction', 'copy')} {r.get('Bytes', '')}B"))
    api = []
    for r in rows(d, "*hip_api_trace.csv"):
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if b - a > 200_000:
            api.append((a, b, "A", r.get("Function", r.get("Kind", "api"))))
    ev.sort()
    # the last step: from the last rs_sig launch on
    sig = [e for e in ev if e[2] == "K" and "rs_sig" in e[3]]
    t0 = sig[-1][0] if sig else ev[0][0]
    t1 = max(e[1] for e in ev)
    gpu = [e for e in ev if e[0] >= t0]
    allev = sorted(gpu + [a for a in api if a[0] >= t0])
    print(f"last step: {(t1 - t0) / 1e6:.3f} ms from the signatures launch to the last GPU activity")
    busy = 0
    end = t0
    for a, b, k, n in gpu:
        busy += max(0, b - max(a, end))
        end = max(end, b)
    print(f"GPU busy {busy / 1e6:.3f} ms, idle {(t1 - t0 - busy) / 1e6:.3f} ms")
    last_end = t0
    for a, b, k, n in allev:
        gap = (a - last_end) / 1e6 if k != "A" else 0.0
        mark = f"  <gap {gap:.3f} ms>" if gap > 0.2 else ""
        print(f"{(a - t0) / 1e6:10.3f} {(b - a) / 1e6:9.3f} {k} {n}{mark}")
        if k != "A":
            last_end = max(last_end, b)


if __name__ == "__main__":
    main()
